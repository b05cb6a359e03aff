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


def _geometry(frames, kw):
    """(scaled W, H, worker kwargs) as the reference derives them (fd:57-61)."""
    kw = dict(kw)
    sf = kw.pop("scale_factor", 1.0)
    H, W = frames.shape[1:3]
    return int(W * sf), int(H * sf), dict(kw, src_width=W, src_height=H)


def _check(name, meta, arrs, frames, ovs, cps):
    m = meta[name]
    assert [_sha(f) for f in frames] == m["input_sha256"], f"{name}: synthetic generator drifted"
    assert len(cps) == m["frames_processed"], (name, len(cps), m["frames_processed"])
    if name in FULL_ARRAYS:
        for t, o in enumerate(ovs):
            assert np.array_equal(o, arrs[f"{name}__overlay"][t]), (name, "overlay", t)
        for t, c in enumerate(cps):
            assert np.array_equal(c, arrs[f"{name}__compressed"][t]), (name, "compressed", t)
    assert [_sha(o) for o in ovs] == m["overlay_sha256"], (name, "overlay")
    assert [_sha(c) for c in cps] == m["compressed_sha256"], (name, "compressed")


@pytest.mark.parametrize("name", list(CASES))
def test_oracle_reproduces_reference(oracle_lib, golden, name):
    meta, arrs = golden
    mk, kw = CASES[name]
    frames = mk()
    W, H, wkw = _geometry(frames, kw)
    ref = oracle_lib.OracleFD(W, H, **wkw)
    ref.prime(frames[0])
    ovs, cps = [], []
    for f in frames[1:]:
        try:
            o, c, _ = ref.step(f)
        except oracle_lib.OddDCTError as e:     # the reference's loop ends here (fd:122, fd:140)
            ovs.append(e.overlay)
            break
        ovs.append(o)
        cps.append(c)
    assert ref.stats()["frames"] == len(cps)
    _check(name, meta, arrs, frames, ovs, cps)


@pytest.mark.gpu
@pytest.mark.parametrize("name", list(CASES))
def test_hip_reproduces_reference(gpu_lib, golden, name):
    """Per-frame steps, then the same clip as one batch (max_batch 4)."""
    from dvc_amd._native import DVC_E_ODD_DCT, DvcError
    meta, arrs = golden
    mk, kw = CASES[name]
    frames = mk()
    W, H, wkw = _geometry(frames, kw)
    w = gpu_lib.FDWorker(W, H, **wkw)
    w.prime(frames[0])
    ovs, cps = [], []
    for f in frames[1:]:
        ov, cp = np.empty((H, W, 3), np.uint8), np.empty((H, W, 3), np.uint8)
        try:
            w.step(f, ov, cp)
        except DvcError as e:
            assert e.code == DVC_E_ODD_DCT, e
            ovs.append(ov)
            break
        ovs.append(ov)
        cps.append(cp)
    assert w.stats()["frames"] == len(cps)
    w.close()
    _check(name, meta, arrs, frames, ovs, cps)
    # batched: frames [0, k) complete, overlay k valid, stats count k
    w = gpu_lib.FDWorker(W, H, max_batch=4, **wkw)
    w.prime(frames[0])
    ov = np.empty((len(frames) - 1, H, W, 3), np.uint8)
    cp = np.empty_like(ov)
    try:
        w.step_batch(frames[1:], ov, cp)
    except DvcError as e:
        assert e.code == DVC_E_ODD_DCT, e
    k = w.stats()["frames"]
    w.close()
    _check(name, meta, arrs, frames, list(ov[:min(k + 1, len(ov))]), list(cp[:k]))
