"""Wide frames and the create-time range checks (GPU).

* OF at 8320 px: k_pyr_h stages a source row in LDS — as floats,
  double-buffered, up to 8 KB rows; wider rows as their bytes, single-buffered
  (of_kernels.hip PH_F32_LDS). 8320 x 112 has one pyramid level, so the byte
  form runs; flow, masks and compressed frames bit-exact vs the oracle.
* FD at 8320 px through the fused front, vs the oracle.
* Values the GPU path cannot take are refused at create with
  DVC_E_UNSUPPORTED (never a launch failure later): FD rows beyond the
  contour filter's LDS row index (~32k px), block_size > 128, kernel_size
  > 127; OF window_size > 255, morph_kernel > 64.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _wide(seed, n=3):
    """8320 x 112: 13 copies of a 640 x 112 clip side by side (the generator's
    objects scale with the width and would not fit 112 rows)."""
    from dvc_amd.synthetic import clip
    return np.ascontiguousarray(np.tile(clip(640, 112, n, seed=seed, n_objects=3), (1, 1, 13, 1)))


def test_of_wide_frame(gpu_lib, oracle_lib):
    from tests.test_of_gpu import _run_pair
    _run_pair(gpu_lib, oracle_lib, _wide(31))


def test_fd_wide_frame(gpu_lib, oracle_lib):
    from tests.test_fd_gpu import _run_pair
    _run_pair(gpu_lib, oracle_lib, _wide(32))


@pytest.mark.parametrize("kw", [
    {"width": 40000, "height": 64},
    {"block_size": 130},
    {"kernel_size": 128},
])
def test_fd_refused_at_create(gpu_lib, kw):
    from dvc_amd._native import DVC_E_UNSUPPORTED, DvcError
    W, H = kw.pop("width", 640), kw.pop("height", 360)
    with pytest.raises(DvcError) as e:
        gpu_lib.FDWorker(W, H, **kw)
    assert e.value.code == DVC_E_UNSUPPORTED


@pytest.mark.parametrize("kw", [{"window_size": 256}, {"morph_kernel": 65}])
def test_of_refused_at_create(gpu_lib, kw):
    from dvc_amd._native import DVC_E_UNSUPPORTED, DvcError
    with pytest.raises(DvcError) as e:
        gpu_lib.OFWorker(640, 360, **kw)
    assert e.value.code == DVC_E_UNSUPPORTED


def test_fd_odd_width_staged_not_overread(gpu_lib, oracle_lib):
    """W % 4 != 0 device frames in a buffer that ends at the frame span (the last
    row's 3W bytes, no padding): read through the staged copy, never in place."""
    import torch
    from dvc_amd.synthetic import clip
    W, H, n = 642, 120, 5
    frames = clip(W, H, n, seed=33, n_objects=3)
    dev = torch.device("cuda", 0)
    seq = torch.from_numpy(frames).to(dev)          # dense: frame span = 3WH, pitch 3W (not a multiple of 4)
    w = gpu_lib.FDWorker(W, H, device_ptrs=True, max_batch=4)
    w.prime(seq[0])
    ov = torch.empty((n - 1, H, W, 3), dtype=torch.uint8, device=dev)
    cp = torch.empty_like(ov)
    w.step_batch(seq[1:], ov, cp)
    w.sync()
    w.close()
    ref = oracle_lib.OracleFD(W, H)
    ref.prime(frames[0])
    for t in range(1, n):
        rov, rcp, _ = ref.step(frames[t])
        assert np.array_equal(ov[t - 1].cpu().numpy(), rov), t
        assert np.array_equal(cp[t - 1].cpu().numpy(), rcp), t
    ref.close()
