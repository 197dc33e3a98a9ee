// Box-Muller for the S4.1 noise (fsf:80-88, the Philox stream of oracle/philox.py): ln(u) for u in
// (0, 1] within 1 ulp and (sin, cos)(2 pi u) for u in [0, 1] within 1.4e-16 absolute, on the
// restricted domains the noise needs -- no special cases, no large-argument reduction, a refined
// reciprocal instead of a division.  The library's general ln / sincos cost k_synth about twice as
// many VALU instructions (profiles/r06t_synth_ablation.txt).  tools/noise_math_check.cpp
// (tests/test_noise_math.py) compares both with long-double libm on the host.
#pragma once
#include <cstdint>

#ifndef RSP_NM
#define RSP_NM __device__ __forceinline__
#endif
#ifndef RSP_NM_RCP
#define RSP_NM_RCP(x) __builtin_amdgcn_rcp(x)   // v_rcp_f64: refined below
#endif

// ln(u), u in (0, 1] a normal double: u = m 2^e, m in [sqrt(1/2), sqrt(2)), f = m - 1 (exact),
// ln(1 + f) = 2 atanh(s), s = f / (2 + f), as f - (f^2/2 - s (f^2/2 + R(s^2))) with the minimax
// R of the classic fdlibm log (|error| < 1 ulp); e ln 2 in two parts.
RSP_NM double rsp_nm_log(double u) {
    const uint64_t b = __builtin_bit_cast(uint64_t, u);
    int e = (int)(b >> 52) - 1023;
    double m = __builtin_bit_cast(double, (b & 0x000FFFFFFFFFFFFFull) | 0x3FF0000000000000ull);   // [1, 2)
    const bool hi = m > 1.4142135623730951;
    m = hi ? 0.5 * m : m;
    e += hi;
    const double f = m - 1.0;
    const double d = 2.0 + f;
    double r = RSP_NM_RCP(d);
    r = __builtin_fma(__builtin_fma(-d, r, 1.0), r, r);
    r = __builtin_fma(__builtin_fma(-d, r, 1.0), r, r);
    double s = f * r;
    s = __builtin_fma(__builtin_fma(-d, s, f), r, s);
    const double z = s * s, w = z * z;
    const double t1 = w * (3.999999999940941908e-01 + w * (2.222219843214978396e-01 + w * 1.531383769920937332e-01));
    const double t2 = z * (6.666666666666735130e-01 +
                           w * (2.857142874366239149e-01 + w * (1.818357216161805012e-01 + w * 1.479819860511658591e-01)));
    const double R = t2 + t1;
    const double hfsq = 0.5 * f * f;
    const double de = (double)e;
    return de * 6.93147180369123816490e-01 - ((hfsq - (s * (hfsq + R) + de * 1.90821492927058770002e-10)) - f);
}

// sin and cos of 2 pi u, u in [0, 1]: q = round(4u) quarter turns, f = u - q/4 in [-1/8, 1/8]
// (exact), x = 2 pi f in [-pi/4, pi/4], then the fdlibm kernels' minimax polynomials.
RSP_NM void rsp_nm_sincos2pi(double u, double* sn, double* cs) {
    const double k = __builtin_rint(4.0 * u);
    const int q = (int)k & 3;
    const double x = (u - 0.25 * k) * 6.283185307179586477;
    const double z = x * x, w = z * z;
    const double rs = 8.33333333332248946124e-03 + z * (-1.98412698298579493134e-04 + z * 2.75573137070700676789e-06) +
                      z * w * (-2.50507602534068634195e-08 + z * 1.58969099521155010221e-10);
    const double sx = x + (z * x) * (-1.66666666666666324348e-01 + z * rs);
    const double rc = z * (4.16666666666666019037e-02 + z * (-1.38888888888741095749e-03 + z * 2.48015872894767294178e-05)) +
                      w * w * (-2.75573143513906633035e-07 + z * (2.08757232129817482790e-09 + z * -1.13596475577881948265e-11));
    const double hz = 0.5 * z, ww = 1.0 - hz;
    const double cx = ww + (((1.0 - ww) - hz) + z * rc);
    const double s0 = (q & 1) ? cx : sx, c0 = (q & 1) ? sx : cx;
    *sn = (q & 2) ? -s0 : s0;
    *cs = ((q + 1) & 2) ? -c0 : c0;
}
