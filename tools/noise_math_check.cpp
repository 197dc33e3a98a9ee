// Host check of csrc/rsp_noise_math.h against long-double libm on the inputs the noise takes:
// u = (x + 0.5) 2^-32 for 32-bit x (every edge word and argv[1] random ones, default 2^25).  Prints the largest error
// in ulps of each function and of glibc's double log / sin(2.0 * M_PI * u) for comparison.
// build: g++ -O2 -std=c++20 tools/noise_math_check.cpp -o /tmp/nmc && /tmp/nmc
#include <cmath>
#include <cstdio>
#include <random>
#include <cstdlib>
#define RSP_NM static inline
#define RSP_NM_RCP(x) ((double)(1.0f / (float)(x)))   // coarser than v_rcp_f64: the refinement must cope
#include "../radar-signal-simulation-and-target-detection_amd/csrc/rsp_noise_math.h"

static double ulp_err(double got, long double ref) {
    const double r = (double)ref;
    const double u = std::nextafter(std::fabs(r), INFINITY) - std::fabs(r);
    return (double)std::fabs((long double)got - ref) / (r == 0 ? 5e-324 : u);
}

int main(int argc, char** argv) {
    const int n_random = argc > 1 ? atoi(argv[1]) : (1 << 25);
    std::mt19937_64 g(20250101);
    double e_log = 0, e_sin = 0, e_cos = 0, l_log = 0, l_sin = 0, l_cos = 0, a_sin = 0, a_cos = 0;
    const long double TWO_PI = 6.283185307179586476925286766559L;
    auto one = [&](uint32_t x) {
        const double u = ((double)x + 0.5) * 2.3283064365386963e-10;
        const long double lr = logl((long double)u);
        e_log = std::fmax(e_log, ulp_err(rsp_nm_log(u), lr));
        l_log = std::fmax(l_log, ulp_err(std::log(u), lr));
        double s, c;
        rsp_nm_sincos2pi(u, &s, &c);
        const long double sr = sinl(TWO_PI * u), cr = cosl(TWO_PI * u);
        e_sin = std::fmax(e_sin, ulp_err(s, sr));
        e_cos = std::fmax(e_cos, ulp_err(c, cr));
        a_sin = std::fmax(a_sin, (double)std::fabs(s - sr));
        a_cos = std::fmax(a_cos, (double)std::fabs(c - cr));
        l_sin = std::fmax(l_sin, (double)std::fabs(std::sin(2.0 * M_PI * u) - sr));
        l_cos = std::fmax(l_cos, (double)std::fabs(std::cos(2.0 * M_PI * u) - cr));
    };
    for (uint32_t x = 0; x < 4096; ++x) { one(x); one(~x); }
    for (int q = 0; q <= 4; ++q)   // quadrant boundaries
        for (int d = -2048; d <= 2048; ++d) one((uint32_t)((uint64_t)q * 0x40000000ull + d));
    for (int i = 0; i < n_random; ++i) one((uint32_t)g());
    printf("rsp_nm_log      max %.3f ulp   (glibc log %.3f ulp)\n", e_log, l_log);
    printf("rsp_nm_sincos2pi sin max %.3f ulp, %.3g abs; cos max %.3f ulp, %.3g abs\n", e_sin, a_sin, e_cos, a_cos);
    printf("glibc sin/cos(2.0 * M_PI * u) abs error: %.3g / %.3g (the argument's rounding)\n", l_sin, l_cos);
    return (e_log < 2.0 && a_sin < 4e-16 && a_cos < 4e-16) ? 0 : 1;
}
