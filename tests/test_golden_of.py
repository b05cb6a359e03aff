"""Replay the OF golden vectors captured from the reference's own two passes
(tests/golden/make_golden_of.py: temporal_smoothing_flow -> compress_with_motion,
motion_compression_opt.py:29-193) through the oracle (CPU) and through the HIP
C-ABI (GPU, per frame and batched). Bit-exact on every mask and compressed frame."""
import hashlib
import json
import os

import numpy as np
import pytest

from tests.golden.cases_of import CASES, FULL_ARRAYS

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")

# oracle kwargs use the reference's kwarg names except the quantiser
_KW = {"flow_threshold", "alpha_fraction", "window_size", "morph_kernel"}


def _sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


@pytest.fixture(scope="module")
def golden():
    with open(os.path.join(GOLD, "of_golden.json")) as f:
        meta = json.load(f)["cases"]
    arrs = dict(np.load(os.path.join(GOLD, "of_golden.npz")))
    return meta, arrs


def _check(name, meta, arrs, frames, masks, cps):
    m = meta[name]
    assert [_sha(f) for f in frames] == m["input_sha256"], f"{name}: synthetic generator drifted"
    if name in FULL_ARRAYS:
        for t, (mk, c) in enumerate(zip(masks, cps)):
            assert np.array_equal(mk, arrs[f"{name}__mask"][t]), (name, "mask", t)
            assert np.array_equal(c, arrs[f"{name}__compressed"][t]), (name, "compressed", t)
    assert [int((mk > 0).sum()) for mk in masks] == m["mask_px"], (name, "mask pixel counts")
    assert [_sha(mk) for mk in masks] == m["mask_sha256"], (name, "mask")
    assert [_sha(c) for c in cps] == m["compressed_sha256"], (name, "compressed")


@pytest.mark.parametrize("name", list(CASES))
def test_oracle_reproduces_reference_of(oracle_lib, golden, name):
    meta, arrs = golden
    mk, kw = CASES[name]
    frames = mk()
    H, W = frames.shape[1:3]
    ref = oracle_lib.OracleOF(W, H, **{k: v for k, v in kw.items() if k in _KW})
    ref.prime(frames[0])
    outs = [ref.step(f) for f in frames[1:]]
    ref.close()
    _check(name, meta, arrs, frames, [o[0] for o in outs], [o[1] for o in outs])


@pytest.mark.gpu
@pytest.mark.parametrize("name", list(CASES))
def test_hip_reproduces_reference_of(gpu_lib, golden, name):
    meta, arrs = golden
    mk, kw = CASES[name]
    frames = mk()
    H, W = frames.shape[1:3]
    w = gpu_lib.OFWorker(W, H, **kw)
    w.prime(frames[0])
    outs = [w.step(f) for f in frames[1:]]
    w.close()
    _check(name, meta, arrs, frames, [o[0] for o in outs], [o[1] for o in outs])


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["of_s320_w4", "of_s640_seed0"])
def test_hip_batched_reproduces_reference_of(gpu_lib, golden, name):
    meta, arrs = golden
    mk, kw = CASES[name]
    frames = mk()
    H, W = frames.shape[1:3]
    w = gpu_lib.OFWorker(W, H, max_batch=3, **kw)
    w.prime(frames[0])
    masks, cps = w.step_batch(frames[1:])
    w.close()
    _check(name, meta, arrs, frames, list(masks), list(cps))
