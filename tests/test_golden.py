"""Replay the golden vectors captured from the reference's own orchestration
(tests/golden/make_golden.py) — through the oracle (CPU) and through the HIP
C-ABI (GPU). Bit-exact on every overlay and compressed frame."""
import hashlib
import json
import os

import numpy as np
import pytest

from tests.golden.cases import CASES, FULL_ARRAYS

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


@pytest.fixture(scope="module")
def golden():
    with open(os.path.join(GOLD, "fd_golden.json")) as f:
        meta = json.load(f)["cases"]
    arrs = dict(np.load(os.path.join(GOLD, "fd_golden.npz")))
    return meta, arrs


def _check(name, meta, arrs, frames, ovs, cps):
    m = meta[name]
    assert [_sha(f) for f in frames] == m["input_sha256"], f"{name}: synthetic generator drifted"
    if name in FULL_ARRAYS:
        for t, (o, c) in enumerate(zip(ovs, cps)):
            assert np.array_equal(o, arrs[f"{name}__overlay"][t]), (name, "overlay", t)
            assert np.array_equal(c, arrs[f"{name}__compressed"][t]), (name, "compressed", t)
    assert [_sha(o) for o in ovs] == m["overlay_sha256"], (name, "overlay")
    assert [_sha(c) for c in cps] == m["compressed_sha256"], (name, "compressed")


@pytest.mark.parametrize("name", list(CASES))
def test_oracle_reproduces_reference(oracle_lib, golden, name):
    meta, arrs = golden
    mk, kw = CASES[name]
    frames = mk()
    H, W = frames.shape[1:3]
    ref = oracle_lib.OracleFD(W, H, **kw)
    ref.prime(frames[0])
    outs = [ref.step(f) for f in frames[1:]]
    _check(name, meta, arrs, frames, [o[0] for o in outs], [o[1] for o in outs])


@pytest.mark.gpu
@pytest.mark.parametrize("name", list(CASES))
def test_hip_reproduces_reference(gpu_lib, golden, name):
    meta, arrs = golden
    mk, kw = CASES[name]
    frames = mk()
    H, W = frames.shape[1:3]
    if W % 4 or H % 4:
        pytest.skip("GPU path needs multiples of 4")
    w = gpu_lib.FDWorker(W, H, **kw)
    w.prime(frames[0])
    outs = [w.step(f) for f in frames[1:]]
    w.close()
    _check(name, meta, arrs, frames, [o[0] for o in outs], [o[1] for o in outs])
