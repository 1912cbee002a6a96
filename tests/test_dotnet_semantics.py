""".NET-semantics assumptions of the oracle, each pinned by a hand-derived expected value (VERDICT r1
item 8).  The reference's C# cannot run here, so these are the places where the oracle
had to decide how .NET 8 evaluates an expression, stated as tests:

1. LINQ ``float[].Sum()`` accumulates in double and narrows once (MipHelpers.cs:785, ``weights.Sum()``;
   .NET 8 System.Linq ``Sum(IEnumerable<float>)`` keeps a ``double`` accumulator).
2. ``Array.BinarySearch(cdf, u)`` + ``~idx - 1`` (MipHelpers.cs:827-832) selects max{i : cdf_i <= u}
   also on an EXACT hit (the search returns the hit's index), so the oracle's linear scan for
   max{i : cdf_i <= u} is the same function for a strictly increasing cdf.
3. ``Vector3.Dot(d, d)`` / ``Vector3.Length()`` (MipHelpers.cs:370, 503) evaluate ((x*x + y*y) + z*z)
   with every product and sum rounded to fp32 (SSE4.1 dpps with mask 0x71 sums lanes pairwise as
   (l0 + l1) + (l2 + l3) with l3 = 0; the scalar fallback is left to right) and no FMA contraction;
   ``Vector3 / float`` divides element-wise (not a multiply by the reciprocal).

Each expected value below is derived step by step in numpy float32 from the C# expression; the
alternative semantics is computed too and shown to give a different answer for the chosen input, so
each test really discriminates.  The GPU samplers/geometry are bit-exact to the oracle
(test_gpu_kernels.py), so these pins carry over to the HIP path.
"""
import numpy as np

f32 = np.float32


def _blur_pdf_cdf(w, padding, double_sum):
    """ResampleAlongRay blur-pool (MipHelpers.cs:645-661) then SortedPiecewiseConstantPDF steps 1-3
    (MipHelpers.cs:783-810), in fp32 with the chosen Sum semantics."""
    B = len(w)
    wmax = [max(w[0] if i == 0 else w[i - 1], w[B - 1] if i == B else w[i]) for i in range(B + 1)]
    wb = [f32(f32(f32(0.5) * f32(wmax[i] + wmax[i + 1])) + f32(padding)) for i in range(B)]
    if double_sum:
        wsum = f32(sum(float(x) for x in wb))  # double accumulator, one narrowing
    else:
        wsum = f32(0)
        for x in wb:
            wsum = f32(wsum + x)
    pad = max(f32(0), f32(f32(1e-5) - wsum))
    if pad > 0:
        per = f32(pad / f32(B))
        wb = [f32(x + per) for x in wb]
        wsum = f32(wsum + pad)
    cdf = [f32(0)]
    run = f32(0)
    for i in range(B - 1):
        run = f32(run + f32(wb[i] / wsum))
        cdf.append(min(f32(1), run))
    cdf.append(f32(1))
    return cdf


def _sample(t_in, cdf, u):
    idx = max(i for i in range(len(cdf) - 1) if cdf[i] <= u)
    denom = f32(cdf[idx + 1] - cdf[idx])
    t = f32(f32(u - cdf[idx]) / denom) if denom > 0 else f32(0)
    t = min(max(t, f32(0)), f32(1))
    return idx, f32(t_in[idx] + f32(t * f32(t_in[idx + 1] - t_in[idx])))


def _linspace_u(n):
    # D24 (randomized = false): u = linspace(0, 1 - 1e-7, n) as s * ((1 - 1e-7) / (n - 1)) in fp32
    step = f32(f32(f32(1) - f32(1e-7)) / f32(n - 1))
    return [f32(f32(s) * step) for s in range(n)]


def test_linq_float_sum_accumulates_in_double(oracle):
    B, S_out = 64, 64
    t_in = np.linspace(2, 6, B + 1, dtype=np.float32)
    w = np.zeros(B, np.float32)
    w[::7] = np.float32(0.3)  # blur-pooled weights whose fp32 running sum rounds differently
    u = _linspace_u(S_out + 1)
    got_t, got_idx = oracle.sample_pdf(t_in[None], w[None], S_out, 0.01, False)
    exp_d = [_sample(t_in, _blur_pdf_cdf(w, 0.01, True), x) for x in u]
    exp_f = [_sample(t_in, _blur_pdf_cdf(w, 0.01, False), x) for x in u]
    assert [t for _, t in exp_d] != [t for _, t in exp_f], "input does not discriminate the two semantics"
    assert np.array_equal(got_t[0], np.array([t for _, t in exp_d], np.float32))
    assert np.array_equal(got_idx[0], np.array([i for i, _ in exp_d], np.int32))


def test_binary_search_exact_hit_selects_the_hit(oracle):
    """u_s lands exactly on cdf_j: Array.BinarySearch returns j, t = t_in[j] exactly."""
    B, S_out = 2, 2
    u = _linspace_u(S_out + 1)  # [0, (1 - 1e-7)/2, 1 - 1e-7]
    t_in = np.array([2.0, 3.0, 5.0], np.float32)
    # find weights whose cdf_1 = pdf_0 equals u_1 bit for bit: w = [a, 1] with a searched near 1
    hit = None
    a = f32(1.0)
    for _ in range(200000):
        cdf = _blur_pdf_cdf(np.array([a, 1.0], np.float32), 0.0, True)
        if cdf[1] == u[1]:
            hit = a
            break
        a = np.nextafter(a, f32(0)) if cdf[1] > u[1] else np.nextafter(a, f32(2))
    assert hit is not None, "no exact-hit weights found"
    w = np.array([hit, 1.0], np.float32)
    cdf = _blur_pdf_cdf(w, 0.0, True)
    assert cdf[1] == u[1]
    got_t, got_idx = oracle.sample_pdf(t_in[None], w[None], S_out, 0.0, False)
    # C#: BinarySearch finds index 1 (exact), t = (u - cdf1) / (cdf2 - cdf1) = 0 -> t_in[1]
    assert got_idx[0, 1] == 1 and got_t[0, 1] == t_in[1]
    # and u_0 = 0 = cdf_0: the exact hit at index 0 gives t_in[0]
    assert got_idx[0, 0] == 0 and got_t[0, 0] == t_in[0]


def _cov_x(d, tvar, rvar, dms):
    dd = f32(d[0] * d[0])
    return f32(f32(tvar * dd) + f32(rvar * f32(f32(1) - f32(dd / dms))))


def _frustum(t0, t1, radius):
    """t_var, r_var of ConicalFrustumToGaussian (MipHelpers.cs:391-402) in its fp32 op order."""
    mu, hw = f32(f32(t0 + t1) / f32(2)), f32(f32(t1 - t0) / f32(2))
    mu2, hw2 = f32(mu * mu), f32(hw * hw)
    den = f32(f32(f32(3) * mu2) + hw2)
    tvar = f32(f32(hw2 / f32(3)) - f32(f32(f32(f32(4) / f32(15)) * f32(f32(hw2 * hw2) * f32(f32(f32(12) * mu2) - hw2)))
                                      / f32(den * den)))
    r2 = f32(radius * radius)
    rvar = f32(r2 * f32(f32(f32(mu2 / f32(4)) + f32(f32(f32(5) / f32(12)) * hw2))
                        - f32(f32(f32(f32(4) / f32(15)) * f32(hw2 * hw2)) / den)))
    return tvar, rvar


def test_vector3_dot_and_length_order(oracle):
    t0, t1, radius = f32(2.0), f32(2.5), f32(0.003)
    tvar, rvar = _frustum(t0, t1, radius)
    # a direction where ((x^2 + y^2) + z^2) != (x^2 + (y^2 + z^2)) in fp32, and where that 1-ulp
    # difference survives both into the covariance and through sqrtf into Length()
    rng = np.random.default_rng(0)
    for _ in range(100000):
        d = rng.normal(size=3).astype(np.float32)
        sq = [f32(c * c) for c in d]
        left = f32(f32(sq[0] + sq[1]) + sq[2])
        right = f32(sq[0] + f32(sq[1] + sq[2]))
        if (left != right and _cov_x(d, tvar, rvar, left) != _cov_x(d, tvar, rvar, right)
                and np.sqrt(left) != np.sqrt(right)):
            break
    else:
        raise AssertionError("no discriminating direction found")
    # LiftGaussian's directionMagnitudeSquared (MipHelpers.cs:370) -> the covariance, bit for bit
    mean, cov = oracle.cast(np.array([[t0, t1]], np.float32), np.zeros((1, 3), np.float32), d[None],
                            np.array([radius], np.float32))
    assert cov[0, 0, 0] == _cov_x(d, tvar, rvar, left)
    # Vector3.Length() = MathF.Sqrt(Dot) (MipHelpers.cs:503): the alpha of a one-sample ray,
    # 1 - exp(-sigma * delta * |d|) with |d| an fp32 (the oracle's render runs in double after it)
    sigma = 0.01
    C, wts = oracle.render(np.array([[sigma]]), np.zeros((1, 1, 3)), np.array([[0.0, 1.0]], np.float32), d[None],
                           white=False)
    exp_w = 1.0 - np.exp(-sigma * float(np.sqrt(left)))
    assert exp_w != 1.0 - np.exp(-sigma * float(np.sqrt(right)))
    assert wts[0, 0] == exp_w
