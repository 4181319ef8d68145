"""The digit-slice arithmetic of the int8 exact passes (irls_oz_impl.hpp,
wide_oz.hip), restated in numpy on the CPU: the one-FMA
rounding against 1.5 2^52 + 0x8080808080, the five balanced byte digits, the
int32 bounds of the level sums at 32767 rows, and the error of the five kept
levels against the fp64 X^T W X.  (The GPU kernels are checked against the fp64
pass in tests/test_gpu_ozaki.py.)"""

import numpy as np

MAGIC = 6755399441055744.0 + 551911719040.0   # 1.5 2^52 + 0x8080808080
B = 0x8080808080


def digits(z, E):
    """Balanced digits d_0 (top) .. d_4 of F = round(z 2^(38 - E)) as the
    kernels form them: t = fma(z, 2^(38-E), MAGIC); bytes of the low 40 bits
    XOR 0x80."""
    t = z * np.ldexp(1.0, 38 - E) + MAGIC    # exact: |z 2^(38-E)| < 2^38, ulp(t) = 1
    bits = t.view(np.uint64) & np.uint64((1 << 40) - 1)
    d = np.empty(z.shape + (5,), dtype=np.int64)
    for s in range(5):  # s = 0 top digit (bits 32-39) .. 4 (bits 0-7)
        byte = (bits >> np.uint64(8 * (4 - s))) & np.uint64(0xFF)
        d[..., s] = (byte ^ np.uint64(0x80)).astype(np.int64)
        d[..., s] = np.where(d[..., s] >= 128, d[..., s] - 256, d[..., s])
    F = np.round(z * np.ldexp(1.0, 38 - E)).astype(np.int64)
    return d, F


def test_digits_reassemble_the_rounded_value():
    rs = np.random.RandomState(0)
    E = 3
    z = (rs.rand(20000) * 2 - 1) * (2.0 ** E) * 0.999
    d, F = digits(z, E)
    recon = sum(d[:, s] << (8 * (4 - s)) for s in range(5))
    assert np.array_equal(recon, F)
    assert np.abs(d[:, 0]).max() <= 64          # |F| < 2^38: the top digit stays in [-64, 64]
    assert np.abs(d).max() <= 128


def test_level_sums_fit_int32_at_32767_rows():
    # worst case per row: level 4 = 2 x 64 x 128 (d0 d4, d4 d0) + 3 x 128^2 = 2^16
    assert 2 * 64 * 128 + 3 * 128 * 128 == 1 << 16
    assert (1 << 16) * 32767 < 2 ** 31


def test_five_levels_error_against_fp64():
    rs = np.random.RandomState(1)
    n, P = 4000, 12
    X = rs.rand(n, P) - 0.5
    w = rs.rand(n) * 0.25
    z = X * np.sqrt(w)[:, None]
    E = np.frexp(np.abs(z).max(0))[1]            # |z_f| < 2^E_f
    D = np.stack([digits(z[:, f], E[f])[0] for f in range(P)], axis=1)  # [n, P, 5]
    H = np.zeros((P, P))
    for i in range(P):
        for j in range(P):
            L = [sum(int((D[:, i, a] * D[:, j, k - a]).sum()) for a in range(k + 1)
                     if a < 5 and k - a < 5) for k in range(5)]
            H[i, j] = np.ldexp(sum(L[k] * 2.0 ** (-8 * k) for k in range(5)), E[i] + E[j] - 12)
    ref = z.T @ z
    assert np.abs(H - ref).max() / np.abs(ref).max() < 1e-11
    assert np.allclose(H, H.T, rtol=0, atol=0)  # the level sums are symmetric exactly
