"""CPU tests of the oracle (the checker): known answers for every primitive of
frame_differencing.py:74-130, independent scipy formulations, and the literal
Suzuki-Abe path vs the pixel formulation of the contour filter."""
import numpy as np
import pytest
from scipy import fft, ndimage


def test_gaussian_taps(oracle_lib):
    O = oracle_lib
    # fd:93 — GaussianBlur((5,5), 0): OpenCV's binomial table in Q8
    assert O.gauss_taps_q8(5, 0.0).tolist() == [16, 64, 96, 64, 16]
    assert O.gauss_taps_q8(3, 0.0).tolist() == [64, 128, 64]
    # fd:77 — GaussianBlur((25,25), 30): getGaussianKernelBitExact + error diffusion
    k = O.gauss_taps_q8(25, 30.0)
    assert k.sum() == 256
    assert k.tolist() == [10, 10, 10, 10, 10, 10, 10, 11, 10, 11, 10, 11, 10, 11, 10, 11, 10, 11, 10, 10, 10,
                          10, 10, 10, 10]
    for n, s in [(7, 1.5), (9, 0), (15, 2.0), (63, 10.0)]:
        t = O.gauss_taps_q8(n, s)
        assert t.sum() == 256 and (t == t[::-1]).all()


def test_gray_known_answers(oracle_lib):
    px = np.array([[[255, 0, 0], [0, 255, 0], [0, 0, 255], [255, 255, 255], [0, 0, 0], [10, 200, 30]]],
                  np.uint8)
    g = oracle_lib.bgr2gray(px)[0]
    exp = [(b * 1868 + gg * 9617 + r * 4899 + 8192) >> 14 for b, gg, r in px[0].tolist()]
    assert g.tolist() == exp == [29, 150, 76, 255, 0, 128]


def test_blur5_impulse_and_constant(oracle_lib):
    img = np.zeros((11, 11), np.uint8)
    img[5, 5] = 255
    out = oracle_lib.gaussian_blur(img, 5, 0.0)
    k = np.array([1, 4, 6, 4, 1])
    exp = (np.outer(k, k) * 255 + 128) >> 8
    assert (out[3:8, 3:8] == exp).all() and out.sum() == exp.sum()
    c = np.full((20, 30), 77, np.uint8)
    assert (oracle_lib.gaussian_blur(c, 5, 0.0) == 77).all()
    assert (oracle_lib.gaussian_blur(c, 25, 30.0) == 77).all()


def test_blur_reflect101_border(oracle_lib):
    rng = np.random.default_rng(0)
    img = rng.integers(0, 256, (9, 13), dtype=np.uint8)
    out = oracle_lib.gaussian_blur(img, 5, 0.0)
    pad = np.pad(img.astype(np.int64), 2, mode="reflect")  # numpy 'reflect' == OpenCV REFLECT_101
    k = np.array([1, 4, 6, 4, 1])
    h = sum(k[j] * pad[:, j:j + 13] for j in range(5))
    v = sum(k[i] * h[i:i + 9, :] for i in range(5))
    assert (out == (v + 128) >> 8).all()


def test_contour_area_rectangles(oracle_lib):
    for w, h in [(1, 1), (1, 7), (5, 1), (2, 2), (10, 4), (23, 23)]:
        m = np.zeros((40, 40), np.uint8)
        m[5:5 + h, 7:7 + w] = 255
        cs = oracle_lib.find_external_contours(m)
        assert len(cs) == 1
        assert oracle_lib.contour_area2(cs[0]) == 2 * (w - 1) * (h - 1)


def test_contour_filter_keeps_strictly_greater(oracle_lib):
    m = np.zeros((60, 60), np.uint8)
    m[2:23, 2:27] = 255      # area (25-1)*(21-1) = 480
    m[30:52, 30:57] = 255    # area 26*21 = 546
    for lit in (False, True):
        out = oracle_lib.contour_filter(m, 2 * 500, literal=lit)[0]
        assert out[2:23, 2:27].max() == 0 and (out[30:52, 30:57] == 255).all()
        out = oracle_lib.contour_filter(m, 2 * 480, literal=lit)[0]   # 480 > 480 is false
        assert out[2:23, 2:27].max() == 0
        out = oracle_lib.contour_filter(m, 2 * 479, literal=lit)[0]
        assert (out[2:23, 2:27] == 255).all()


def test_contour_filter_fills_holes_and_nested(oracle_lib):
    m = np.zeros((50, 50), np.uint8)
    m[5:45, 5:45] = 255
    m[10:40, 10:40] = 0           # hole
    m[20:30, 20:30] = 255         # nested component in the hole
    m[24:26, 24:26] = 0           # hole in the nested one
    for lit in (False, True):
        out, n = oracle_lib.contour_filter(m, 0, literal=lit)[:2]
        assert n == 1
        assert (out[5:45, 5:45] == 255).all() and out.sum() == 255 * 40 * 40


@pytest.mark.parametrize("seed", range(4))
def test_literal_equals_pixel_formulation(oracle_lib, seed):
    rng = np.random.default_rng(seed)
    for _ in range(150):
        H, W = (int(v) for v in rng.integers(2, 48, 2))
        m = (rng.random((H, W)) < rng.uniform(0.05, 0.95)).astype(np.uint8) * 255
        if rng.random() < 0.3:  # smoother blobs with holes
            m = (ndimage.uniform_filter(m.astype(float), 3) > 127).astype(np.uint8) * 255
        ma2 = int(rng.integers(-1, 80))
        a, na, filled = oracle_lib.contour_filter(m, ma2)
        b, nb = oracle_lib.contour_filter(m, ma2, literal=True)
        assert na == nb and np.array_equal(a, b), (seed, H, W, ma2)


def test_pixel_formulation_vs_scipy(oracle_lib):
    """Independent: ndimage.binary_fill_holes (4-connected background) + 8-connected labels."""
    rng = np.random.default_rng(7)
    for _ in range(40):
        H, W = (int(v) for v in rng.integers(4, 60, 2))
        m = rng.random((H, W)) < rng.uniform(0.1, 0.8)
        _, n, filled = oracle_lib.contour_filter(m.astype(np.uint8) * 255, 0)
        f = ndimage.binary_fill_holes(m)
        assert np.array_equal(filled > 0, f)
        lab, nl = ndimage.label(f, structure=np.ones((3, 3)))
        assert n == nl
        # 2*area from 2x2 windows == literal shoelace of each external contour
        out_all = oracle_lib.contour_filter(m.astype(np.uint8) * 255, -1)[0]
        assert np.array_equal(out_all > 0, f)


def test_dilate_vs_scipy(oracle_lib):
    rng = np.random.default_rng(1)
    m = (rng.random((37, 53)) < 0.05).astype(np.uint8) * 255
    for k in (1, 3, 7, 10):
        a = k // 2
        got = oracle_lib.dilate(m, k)
        # out(x) = max src(x + i - a), i in [0,k): a window [x-a, x+k-1-a]
        exp = ndimage.maximum_filter(m, size=k, mode="constant", cval=0, origin=(k - 1) // 2 - a if k % 2 == 0 else 0)
        if k % 2 == 0:
            exp = np.zeros_like(m)
            for dy in range(-a, k - a):
                for dx in range(-a, k - a):
                    sh = np.zeros_like(m)
                    ys, yd = (slice(dy, None), slice(0, -dy or None)) if dy >= 0 else (slice(0, dy), slice(-dy, None))
                    xs, xd = (slice(dx, None), slice(0, -dx or None)) if dx >= 0 else (slice(0, dx), slice(-dx, None))
                    sh[yd, xd] = m[ys, xs]
                    exp = np.maximum(exp, sh)
        assert np.array_equal(got, exp), k


def test_add_weighted_decay(oracle_lib):
    """fd:107 at release_factor 0.5: 255 decays 128, 64, ..., 1, 0 (0.5 rounds to even)."""
    a = np.array([255], np.uint8)
    z = np.array([0], np.uint8)
    seq = []
    for _ in range(9):
        a = oracle_lib.add_weighted(a, 0.5, z, 0.5, 0.0)
        seq.append(int(a[0]))
    assert seq == [128, 64, 32, 16, 8, 4, 2, 1, 0]
    assert int(oracle_lib.add_weighted(np.array([0], np.uint8), 0.5, np.array([255], np.uint8), 0.5, 0.0)[0]) == 128


def test_ycrcb_roundtrip_gray(oracle_lib):
    """Static FD blocks set Cr = Cb = 128, which maps back to (Y, Y, Y) exactly."""
    y = np.arange(256, dtype=np.uint8)
    ycc = np.stack([y, np.full(256, 128, np.uint8), np.full(256, 128, np.uint8)], -1)[None]
    bgr = oracle_lib.ycrcb2bgr(ycc)[0]
    assert (bgr == y[:, None]).all()


def test_block_dct_vs_scipy(oracle_lib):
    rng = np.random.default_rng(3)
    for B in (4, 8):
        M = oracle_lib.dct_matrix(B).astype(np.float64)
        ref = fft.dct(np.eye(B), norm="ortho", axis=0)
        assert np.allclose(M, ref, atol=1e-6)
        for _ in range(50):
            blk = rng.integers(0, 256, (B, B), dtype=np.uint8)
            got = oracle_lib.block_quant(blk, 100.0)
            d = fft.dctn(blk.astype(np.float64) - 128, norm="ortho")
            q = np.round(d / 100) * 100
            exp = np.clip(fft.idctn(q, norm="ortho") + 128, 0, 255)
            # fp32 vs fp64: identical except where a coefficient sits on a .5 tie
            # or the reconstruction straddles an integer (reported, not hidden)
            assert np.abs(got.astype(float) - np.floor(exp + 1e-9)).max() <= 1 or \
                np.any(np.isclose(np.abs(d / 100) % 1, 0.5, atol=1e-4))


def test_block_dct_dc_only_exact(oracle_lib):
    """A flat block keeps only DC: Y' = trunc(round_half_even(4(v-128)/100)*100/4 + 128) at B=4."""
    for v in range(256):
        blk = np.full((4, 4), v, np.uint8)
        dc = 4.0 * (v - 128)
        q = np.round(np.float32(dc) / np.float32(100)) * 100
        exp = int(np.clip(np.float32(q) * np.float32(0.25) + 128, 0, 255))
        assert oracle_lib.block_quant(blk, 100.0)[0, 0] == exp
