"""Checkpoint / resume of a feed (the per-feed state is the
previous gray and the accumulated mask for FD, fd:107,133; the previous gray
and the 30-mask deque for OF, of:61,84,101): a handle resumed with
dvc_*_set_state from the planes another handle exported continues exactly as
the uninterrupted run — bit for bit, batched or per frame."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("W,H,kw", [(640, 360, {}), (641, 361, {}), (960, 540, dict(block_size=8, kernel_size=10,
                                                                                       release_factor=0.3))])
def test_fd_resume(gpu_lib, W, H, kw):
    from dvc_amd.synthetic import clip
    N = gpu_lib._native
    frames = clip(W, H, 21, seed=W, noisy=True)
    a = gpu_lib.FDWorker(W, H, keep_planes=True, max_batch=4, **kw)
    a.prime(frames[0])
    k = 9
    first = a.step_batch(frames[1:k + 1])
    gray, acc = a.plane(N.PLANE_GRAY), a.plane(N.PLANE_ACC)
    st_k = a.stats()
    rest = a.step_batch(frames[k + 1:])
    st_end = a.stats()
    a.close()
    assert len(first[0]) == k
    b = gpu_lib.FDWorker(W, H, keep_planes=True, max_batch=3, **kw)
    b.set_state(gray, acc)
    got = b.step_batch(frames[k + 1:])
    for t in range(len(rest[0])):
        assert np.array_equal(got[0][t], rest[0][t]), f"overlay differs at frame {k + 1 + t}"
        assert np.array_equal(got[1][t], rest[1][t]), f"compressed differs at frame {k + 1 + t}"
    st_b = b.stats()
    assert st_b == {q: st_end[q] - st_k[q] for q in st_b}, (st_b, st_end, st_k)
    b.close()


@pytest.mark.parametrize("W,H,window", [(320, 176, 4), (170, 100, 30)])
def test_of_resume(gpu_lib, W, H, window):
    from dvc_amd.synthetic import clip
    N = gpu_lib._native
    frames = clip(W, H, 12, seed=W, n_objects=4)
    a = gpu_lib.OFWorker(W, H, keep_planes=True, window_size=window, alpha_fraction=0.4)
    a.prime(frames[0])
    raw, k = [], 7
    for t in range(1, k + 1):
        a.step(frames[t])
        raw.append(a.plane(N.OF_PLANE_RAW))
    gray = a.plane(N.OF_PLANE_GRAY)
    want = [a.step(f) + (a.flow(),) for f in frames[k + 1:]]
    a.close()
    b = gpu_lib.OFWorker(W, H, keep_planes=True, window_size=window, alpha_fraction=0.4, max_batch=2)
    b.set_state(gray, np.stack(raw))
    for i, f in enumerate(frames[k + 1:]):
        mk, cp = b.step(f)
        assert np.array_equal(b.flow().view(np.uint32), want[i][2].view(np.uint32)), f"flow differs at {k + 1 + i}"
        assert np.array_equal(mk, want[i][0]), f"mask differs at frame {k + 1 + i}"
        assert np.array_equal(cp, want[i][1]), f"compressed differs at frame {k + 1 + i}"
    b.close()
