// rsp_kernels.hip -- CDNA4 (gfx950) kernels of the per-frame radar chain.
//
// Pipeline per frame (all linear stages reordered so every stage streams its
// natural axis):
//   k1_dbf_mtd  : cube [C][N][P] (MATLAB [P x N x C], pulse fastest) -> for each used
//                 fast-time sample n: DBF over channels (fsf:93-97, y = x * W'),
//                 MTD window + P-point FFT + fftshift over pulses (fsf:131-136);
//                 writes Doppler-domain rows z[b][tile][v][NT] (NT samples per 64 B).
//   k2_pc       : pulse compression along fast time of every (beam, Doppler) row
//                 (fsf:101-126): direct FIR for the narrow segment, overlap-save FFT
//                 (Stockham radix-16/8/4/2 in LDS) for medium/long, gate stitching
//                 fused into the output store -> RDM [B][P][G] + |RDM|.
//   k3_cfar     : |RDM| adjacent-beam sum (fsf:184-187), cross GOCA-CFAR (fsf:192-213),
//                 atomic compaction (fsf:215-221) and S9 spline/monopulse estimation
//                 (fsf:237-290) of each detection.
//   k_mtd_cols  : MTD over pulses of a pulse-compressed cube (stage-2 path).
//   k_synth     : S4 echo synthesis + S4.1 Philox noise (fsf:45-88) on the device.
//
// Every kernel is a template over the real type T of the plan: double (complex128, the
// reference's MATLAB arithmetic; the default) or float (complex64).  Complex values are
// 2-wide ext_vector pairs (re, im) of T in registers, LDS and HBM alike.
#include "rsp_internal.h"
#include "rsp_noise_math.h"
#include <math.h>
#include <algorithm>

namespace {

typedef float f2 __attribute__((ext_vector_type(2)));
typedef double d2 __attribute__((ext_vector_type(2)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef double f64x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

template <class T> struct CxT;
template <> struct CxT<float> { typedef f2 V; };
template <> struct CxT<double> { typedef d2 V; };
template <class T> using cx = typename CxT<T>::V;   // complex of T
template <class V> struct ScalT;
template <> struct ScalT<f2> { typedef float S; };
template <> struct ScalT<d2> { typedef double S; };
template <class V> using scal = typename ScalT<V>::S;

// ---- complex arithmetic ------------------------------------------------------------------
// float: complex adds are single v_pk_add_f32 and products two packed ops; double: plain
// v_fma_f64 (gfx950 has no packed f64 arithmetic).
__device__ __forceinline__ f2 vmul(f2 a, f2 b) { return a.xx * b + a.yy * f2{-b.y, b.x}; }
__device__ __forceinline__ d2 vmul(d2 a, d2 b) { return d2{a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x}; }
template <bool INV>
__device__ __forceinline__ f2 vrot(f2 a) {   // * (-i) forward, * (+i) inverse
    return INV ? a.yx * f2{-1.f, 1.f} : a.yx * f2{1.f, -1.f};
}
template <bool INV>
__device__ __forceinline__ d2 vrot(d2 a) {
    return INV ? d2{-a.y, a.x} : d2{a.y, -a.x};
}
template <bool INV, class V>
__device__ __forceinline__ V vtw(double c, double s) {   // exp(-+ i theta)
    typedef scal<V> S;
    return V{(S)c, (S)(INV ? s : -s)};
}
// |x| (fsf:184-185 abs): hardware square root for float (v_sqrt_f32, 1 ulp); for double the
// compiler's own refinement of v_rsq_f64 (Goldschmidt step + two Newton corrections) without
// its ldexp scaling and class checks, which guard only denormal / infinite inputs -- not the
// magnitudes of a radar map; 0 stays 0.
__device__ __forceinline__ float cmag(f2 x) { return __builtin_amdgcn_sqrtf(x.x * x.x + x.y * x.y); }
__device__ __forceinline__ double cmag(d2 x) {
    const double q = x.x * x.x + x.y * x.y;
    const double r = __builtin_amdgcn_rsq(q);           // v_rsq_f64
    double g = q * r, h = 0.5 * r;
    const double r0 = __builtin_fma(-h, g, 0.5);
    g = __builtin_fma(g, r0, g);
    h = __builtin_fma(h, r0, h);
    g = __builtin_fma(__builtin_fma(-g, g, q), h, g);
    g = __builtin_fma(__builtin_fma(-g, g, q), h, g);
    return q > 0.0 ? g : 0.0;
}

// Raw buffer resources (SRSRC): 32-bit byte offsets and hardware range checking.  An offset at
// or past num_records reads 0 / drops the store, so masked lanes need no branch or select.
// The read/write barrier inside an in-place LDS pass (every read of the pass before any write)
#define RSP_WAR_SYNC() __syncthreads()
#define RSP_OOB 0x80000000u   // > any buffer this library makes (plans are validated < 2 GB/frame)
__device__ __forceinline__ __amdgpu_buffer_rsrc_t buf_rsrc(const void* p, unsigned bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, (int)bytes, 0x00020000);
}
// AUX: cache-policy bits of the load (2 = non-temporal)
template <class V, int AUX = 0> __device__ __forceinline__ V buf_ld(__amdgpu_buffer_rsrc_t r, unsigned off) {
    static_assert(sizeof(V) == 8 || sizeof(V) == 16, "one complex sample");
    if constexpr (sizeof(V) == 8)
        return __builtin_bit_cast(V, __builtin_amdgcn_raw_buffer_load_b64(r, (int)off, 0, AUX));
    else
        return __builtin_bit_cast(V, __builtin_amdgcn_raw_buffer_load_b128(r, (int)off, 0, AUX));
}
// A twiddle table in global memory read through a buffer resource: tw + e advances the per-lane
// byte offset, tw[i] (i a constant after unrolling) goes to the instruction's scalar offset, so
// the lgR loads of a butterfly share one offset VGPR instead of a 64-bit address each.
template <class V>
struct TwG {
    __amdgpu_buffer_rsrc_t r;
    unsigned off;
    __device__ __forceinline__ TwG operator+(int e) const { return TwG{r, off + (unsigned)e * (unsigned)sizeof(V)}; }
    __device__ __forceinline__ V operator[](int i) const {
        if constexpr (sizeof(V) == 8)
            return __builtin_bit_cast(V, __builtin_amdgcn_raw_buffer_load_b64(r, (int)off, i * (int)sizeof(V), 0));
        else
            return __builtin_bit_cast(V, __builtin_amdgcn_raw_buffer_load_b128(r, (int)off, i * (int)sizeof(V), 0));
    }
};
// AUX: cache-policy bits of the store (2 = non-temporal)
template <int AUX = 0>
__device__ __forceinline__ void buf_st(__amdgpu_buffer_rsrc_t r, unsigned off, f2 x) {
    __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, x), r, (int)off, 0, AUX);
}
template <int AUX = 0>
__device__ __forceinline__ void buf_st(__amdgpu_buffer_rsrc_t r, unsigned off, d2 x) {
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, x), r, (int)off, 0, AUX);
}
template <int AUX = 0>
__device__ __forceinline__ void buf_st1(__amdgpu_buffer_rsrc_t r, unsigned off, float x) {
    __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(x), r, (int)off, 0, AUX);
}
template <int AUX = 0>
__device__ __forceinline__ void buf_st1(__amdgpu_buffer_rsrc_t r, unsigned off, double x) {
    __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, x), r, (int)off, 0, AUX);
}
// Non-temporal z and RDM stores: z (50 MB per frame, read back by K2 after the whole launch) and
// the RDM (never re-read on the device) only evict lines from L2 and the Infinity Cache
// (interleaved A/B: K1 -5.5 %, k2_pc -1.2 %).
#define RSP_Z_AUX 2     // K1's z stores
#define RSP_RDM_AUX 2   // K2's RDM stores

// Diagnostic builds (-DRSP_DEBUG_KNOBS) only: K2 phase stamps.  Workgroup (f, x) of a k2_pc
// launch writes s_memrealtime (100 MHz) at its phase boundaries into rsp_k2_trace[(f G + x) 8 +
// i], i < 6, plus its job type [6] and hardware position (HW_ID | XCC_ID << 32) [7]
// (tools/ab/k2_phases.py).  The shipped library has neither the variable nor the stamps.
#ifdef RSP_DEBUG_KNOBS
__device__ unsigned long long* rsp_k2_trace;
#define K2_STAMP(i)                                                                                     \
    do {                                                                                                \
        if (rsp_k2_trace && threadIdx.x == 0)                                                           \
            rsp_k2_trace[((size_t)blockIdx.y * gridDim.x + blockIdx.x) * 8 + (i)] = wall_clock64();    \
    } while (0)
#define K2_TAG(v)                                                                                       \
    do {                                                                                                \
        if (rsp_k2_trace && threadIdx.x == 0) {                                                         \
            unsigned long long* t_ = rsp_k2_trace + ((size_t)blockIdx.y * gridDim.x + blockIdx.x) * 8;  \
            t_[6] = (v);                                                                                \
            t_[7] = (unsigned long long)__builtin_amdgcn_s_getreg((31 << 11) | 4) |                     \
                    ((unsigned long long)__builtin_amdgcn_s_getreg((31 << 11) | 20) << 32);             \
        }                                                                                               \
    } while (0)
extern "C" int rsp_debug_set_k2_trace(unsigned long long* p) {
    return (int)hipMemcpyToSymbol(HIP_SYMBOL(rsp_k2_trace), &p, sizeof(p));
}
// persistent K1: workgroup x, loop iteration it < 64 writes [(x 64 + it) 4 + i] (tools/ab/k1_phases.py)
__device__ unsigned long long* rsp_k1_trace;
#define K1_STAMP(it, i)                                                                                 \
    do {                                                                                                \
        if (rsp_k1_trace && threadIdx.x == 0 && (it) < 64)                                              \
            rsp_k1_trace[((size_t)blockIdx.x * 64 + (it)) * 4 + (i)] = wall_clock64();                 \
    } while (0)
extern "C" int rsp_debug_set_k1_trace(unsigned long long* p) {
    return (int)hipMemcpyToSymbol(HIP_SYMBOL(rsp_k1_trace), &p, sizeof(p));
}
#else
#define K2_STAMP(i) ((void)0)
#define K2_TAG(v) ((void)0)
#define K1_STAMP(it, i) ((void)0)
#endif

// ---- radix-R DFT kernels in registers -------------------------------------------------
// Radix-2 butterfly with a twiddle, (a, b) <- (a + w b, a - w b): four FMAs for a + w b and one
// per component for a - w b = 2a - (a + w b) -- 6 operations instead of a complex multiply (4)
// plus an add and a subtract (4).
template <class V>
__device__ __forceinline__ void bfly_tw(V& a, V& b, V w) {
    typedef scal<V> S;
    const V t = a + w.xx * b + w.yy * V{-b.y, b.x};
    b = a * (S)2 - t;
    a = t;
}
template <int R, bool INV, class V> struct Dft;
template <bool INV, class V> struct Dft<2, INV, V> {
    static __device__ __forceinline__ void run(V* a) {
        const V t = a[0];
        a[0] = t + a[1];
        a[1] = t - a[1];
    }
};
template <bool INV, class V> struct Dft<4, INV, V> {
    static __device__ __forceinline__ void run(V* a) {
        const V t0 = a[0] + a[2], t1 = a[0] - a[2];
        const V t2 = a[1] + a[3], t3 = vrot<INV>(a[1] - a[3]);
        a[0] = t0 + t2;
        a[2] = t0 - t2;
        a[1] = t1 + t3;
        a[3] = t1 - t3;
    }
};
template <bool INV, class V> struct Dft<8, INV, V> {
    static __device__ __forceinline__ void run(V* a) {
        V e[4] = {a[0], a[2], a[4], a[6]};
        V o[4] = {a[1], a[3], a[5], a[7]};
        Dft<4, INV, V>::run(e);
        Dft<4, INV, V>::run(o);
        constexpr double r = 0.70710678118654752440;
        o[2] = vrot<INV>(o[2]);
        bfly_tw(e[1], o[1], vtw<INV, V>(r, r));
        bfly_tw(e[3], o[3], vtw<INV, V>(-r, r));
        a[0] = e[0] + o[0];
        a[4] = e[0] - o[0];
        a[2] = e[2] + o[2];
        a[6] = e[2] - o[2];
        a[1] = e[1];
        a[5] = o[1];
        a[3] = e[3];
        a[7] = o[3];
    }
};
template <bool INV, class V> struct Dft<16, INV, V> {
    static __device__ __forceinline__ void run(V* a) {
        V e[8], o[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            e[k] = a[2 * k];
            o[k] = a[2 * k + 1];
        }
        Dft<8, INV, V>::run(e);
        Dft<8, INV, V>::run(o);
        constexpr double c1 = 0.92387953251128675613, s1 = 0.38268343236508977173, r = 0.70710678118654752440;
        o[4] = vrot<INV>(o[4]);
        bfly_tw(e[1], o[1], vtw<INV, V>(c1, s1));
        bfly_tw(e[2], o[2], vtw<INV, V>(r, r));
        bfly_tw(e[3], o[3], vtw<INV, V>(s1, c1));
        bfly_tw(e[5], o[5], vtw<INV, V>(-s1, c1));
        bfly_tw(e[6], o[6], vtw<INV, V>(-r, r));
        bfly_tw(e[7], o[7], vtw<INV, V>(-c1, s1));
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            if (k == 0 || k == 4) {
                a[k] = e[k] + o[k];
                a[k + 8] = e[k] - o[k];
            } else {
                a[k] = e[k];
                a[k + 8] = o[k];
            }
        }
    }
};

// Odd radices of the mixed-radix overlap-save blocks (M = 5 * 2^k, 3 * 2^k).
template <bool INV, class V> struct Dft<3, INV, V> {
    static __device__ __forceinline__ void run(V* a) {
        typedef scal<V> S;
        constexpr double h = 0.86602540378443864676;   // sin(2 pi / 3)
        const V s = a[1] + a[2], d = a[1] - a[2];
        const V t = a[0] - s * (S)0.5;
        const V u = vrot<INV>(d) * (S)h;                // -+ i sin(2pi/3) (x1 - x2)
        a[0] = a[0] + s;
        a[1] = t + u;
        a[2] = t - u;
    }
};
template <bool INV, class V> struct Dft<5, INV, V> {
    static __device__ __forceinline__ void run(V* a) {
        typedef scal<V> S;
        constexpr double c1 = 0.30901699437494742410, c2 = -0.80901699437494742410;   // cos(2pi/5), cos(4pi/5)
        constexpr double s1 = 0.95105651629515357212, s2 = 0.58778525229247312917;    // sin(2pi/5), sin(4pi/5)
        const V a1 = a[1] + a[4], b1 = a[1] - a[4], a2 = a[2] + a[3], b2 = a[2] - a[3];
        const V r1 = a[0] + a1 * (S)c1 + a2 * (S)c2, r2 = a[0] + a1 * (S)c2 + a2 * (S)c1;
        const V u1 = vrot<INV>(b1 * (S)s1 + b2 * (S)s2), u2 = vrot<INV>(b1 * (S)s2 - b2 * (S)s1);
        a[0] = a[0] + a1 + a2;
        a[1] = r1 + u1;
        a[4] = r1 - u1;
        a[2] = r2 + u2;
        a[3] = r2 - u2;
    }
};
// Good-Thomas prime-factor DFT of N = N1 N2 (coprime), no internal twiddles: input n =
// (N2 n1 + N1 n2) mod N, output k = (N2 (N2^-1 mod N1) k1 + N1 (N1^-1 mod N2) k2) mod N.
constexpr int inv_mod(int a, int m) {
    for (int x = 1; x < m; ++x)
        if ((a * x) % m == 1) return x;
    return 1;
}
template <int N1, int N2, bool INV, class V>
__device__ __forceinline__ void dft_pfa(V* a) {
    constexpr int N = N1 * N2;
    V y[N1][N2];
#pragma unroll
    for (int n1 = 0; n1 < N1; ++n1) {
#pragma unroll
        for (int n2 = 0; n2 < N2; ++n2) y[n1][n2] = a[(N2 * n1 + N1 * n2) % N];
        Dft<N2, INV, V>::run(y[n1]);
    }
#pragma unroll
    for (int k2 = 0; k2 < N2; ++k2) {
        V c[N1];
#pragma unroll
        for (int n1 = 0; n1 < N1; ++n1) c[n1] = y[n1][k2];
        Dft<N1, INV, V>::run(c);
#pragma unroll
        for (int k1 = 0; k1 < N1; ++k1)
            a[(N2 * inv_mod(N2 % N1, N1) * k1 + N1 * inv_mod(N1 % N2, N2) * k2) % N] = c[k1];
    }
}
template <bool INV, class V> struct Dft<10, INV, V> {
    static __device__ __forceinline__ void run(V* a) { dft_pfa<2, 5, INV>(a); }
};
template <bool INV, class V> struct Dft<12, INV, V> {
    static __device__ __forceinline__ void run(V* a) { dft_pfa<4, 3, INV>(a); }
};

constexpr int clog2(int x) { return x <= 1 ? 0 : 1 + clog2(x >> 1); }

// LDS index inside a row: SH > 0 inserts one complex every 2^SH to break power-of-two
// strides (tools/ab/lds_conflicts.py models the gfx950 bank rules for each pass).
template <int SH>
__device__ __forceinline__ int lidx(int i) { return SH ? i + (i >> SH) : i; }

// Store policies for the Stockham pass output.  put(idx, row, o, loff, x): idx = t * R + r for
// butterfly t / element r of this thread (a constant after unrolling), row, natural position
// o, and the padded LDS offset loff of (row, o).
template <class V>
struct StoreLds {
    V* buf;
    __device__ __forceinline__ void put(int, int, int, int loff, V x) const { buf[loff] = x; }
};
// A pass whose output goes back into the LDS rows it reads needs the read/write barrier; one
// that stores to global memory (the FFT's last pass into z or the RDM) does not.
template <class St> struct StoresLds { static constexpr bool value = false; };
template <class V> struct StoresLds<StoreLds<V>> { static constexpr bool value = true; };

// Twiddles w[r] = W_{Ns R}^{k r}, r = 1..R-1, of one butterfly (conjugated for the inverse)
// from this pass's table: CMP = false: full rows [k][r-1] (R-1 loads, twk = row k); CMP = true:
// compact columns [i][k] = W^(k 2^i) (lgR loads, twk = table + k, column stride NS), the other
// powers formed as products of at most lgR - 1 of them.  Column-major so that the lanes of a
// pass (consecutive k) read consecutive 16-B entries: conflict-free, where [k][i] rows of 4
// entries put every 4th lane on the same banks (tools/ab/lds_conflicts_k2v2.py).
template <int R, bool INV, bool CMP, int NS, class V, class TW>
__device__ __forceinline__ void load_tw(const TW& twk, V (&w)[R]) {
    if constexpr (!CMP) {
#pragma unroll
        for (int r = 1; r < R; ++r) {
            const V t = twk[r - 1];
            w[r] = V{t.x, INV ? -t.y : t.y};
        }
    } else {
        constexpr int lgR = clog2(R - 1) + 1;   // bases W^(k 2^i), 2^i < R (= log2 R for powers of two)
        V b[lgR];
#pragma unroll
        for (int i = 0; i < lgR; ++i) {
            const V t = twk[i * NS];
            b[i] = V{t.x, INV ? -t.y : t.y};
        }
#pragma unroll
        for (int r = 1; r < R; ++r) {
            const int hb = 1 << clog2(r);
            w[r] = (hb == r) ? b[clog2(r)] : vmul(w[hb], w[r - hb]);
        }
    }
}
constexpr int tw_row(int R, bool cmp) { return cmp ? clog2(R - 1) + 1 : R - 1; }

// Radix plan of a 2^m-point FFT: radix-16 passes, remainder as 8/4 (m = 5 -> 8 x 4);
// must match radix_plan() in rsp_plan.cpp.  REV = the same radices in reverse order (the
// inverse FFT of the overlap-save block, so that its first pass consumes exactly the
// elements the forward FFT's last pass leaves in each thread's registers).
constexpr int rad_bits(int m, int q) {
    for (int i = 0; i < q; ++i) m -= (m == 5) ? 3 : (m >= 4 ? 4 : m);
    return (m == 5) ? 3 : (m >= 4 ? 4 : m);
}
constexpr int n_passes(int m) {
    int n = 0;
    while (m > 0) {
        m -= (m == 5) ? 3 : (m >= 4 ? 4 : m);
        ++n;
    }
    return n;
}
// PAL: the overlap-save blocks' plan puts the smallest radix in the middle of a 3-pass plan
// (2048 = 16 x 8 x 16, 1024 = 16 x 4 x 16): a palindrome, so the inverse FFT runs the same
// radices, and both Ns = 1 passes -- the forward first pass and the inverse first pass fused
// into the forward last one -- are radix 16, whose stride-16 stores are at most 2-way
// conflicted (tools/ab/lds_conflicts64.py).  Must match radix_plan() in rsp_plan.cpp.
constexpr int rad_bits_pal(int m, int q) {
    return n_passes(m) == 3 && q >= 1 ? rad_bits(m, 3 - q) : rad_bits(m, q);
}
constexpr int rad_bits_p(int m, int q, bool rev, bool pal = false) {
    return pal ? (rev ? rad_bits_pal(m, n_passes(m) - 1 - q) : rad_bits_pal(m, q))
               : (rev ? rad_bits(m, n_passes(m) - 1 - q) : rad_bits(m, q));
}

// Offset of pass q's twiddle table inside the concatenated per-pass tables of a 2^LG FFT:
// pass i >= 1 owns Ns_i rows of tw_row(R_i) entries (pass 0: Ns = 1, no twiddles).  Must
// match build_pass_twiddles() in rsp_plan.cpp.
constexpr int tw_pass_off(int LG, int q, bool rev = false, bool cmp = false, bool pal = false) {
    int off = 0, lgns = 0;
    for (int i = 0; i < q; ++i) {
        const int rb = rad_bits_p(LG, i, rev, pal);
        if (i > 0) off += (1 << lgns) * tw_row(1 << rb, cmp);
        lgns += rb;
    }
    return off;
}
constexpr int tw_total(int LG, bool rev = false, bool cmp = false, bool pal = false) {
    return tw_pass_off(LG, n_passes(LG), rev, cmp, pal);
}

// One Stockham radix-R pass (Govindaraju et al. formulation) over `nrows` rows of
// length L = 2^LGL held in LDS (row stride rs).  Ns = 2^LGNS = product of the earlier
// radices.  Reads stride L/R, twiddle W_{Ns R}^{(j mod Ns) r} (from this pass's table),
// radix-R DFT, writes positions expand(j, Ns, R) + r Ns.  In place: all reads, barrier,
// all writes, barrier.  Every size is a compile-time constant, so a pass is straight-line
// code and no address math is carried across passes.
// With power-of-two nb, Ns and pads every 2^SH, lidx(j + r nb) = lidx(j) + r nb + ((r nb) >> SH)
// and lidx(idxD + r Ns) = lidx(idxD) + r Ns + ((r Ns) >> SH): every LDS address of a butterfly
// is a per-thread base plus a compile-time offset (ds_read/ds_write immediate offsets).
template <int R, bool INV, int NB, int SH, int NTHR, int LGL, int LGNS, bool CMP = false, int XL = 0, class V, class TW>
__device__ __forceinline__ void sh_load(const V* buf, int rs, int nrows, const TW& tw, V (&v)[NB][R]) {
    constexpr int lgR = clog2(R);
    constexpr int lgnb = LGL - lgR;
    constexpr int nb = 1 << lgnb;
    constexpr int Ns = 1 << LGNS;
    static_assert(!XL || nb % 128 == 0, "XOR-swizzled input needs r nb to keep the swizzle bits");
    const int total = nb * nrows;
#pragma unroll
    for (int t = 0; t < NB; ++t) {
        const int beta = threadIdx.x + t * NTHR;
        if (beta < total) {
            const int row = beta >> lgnb, j = beta & (nb - 1);
            const int k = j & (Ns - 1);
            const V* src = XL ? buf + (row << LGL) + (j ^ ((j >> 4) & 7)) : buf + row * rs + lidx<SH>(j);
            V w[R];
            if (LGNS > 0) load_tw<R, INV, CMP, Ns>(tw + (CMP ? k : k * tw_row(R, CMP)), w);
#pragma unroll
            for (int r = 0; r < R; ++r) {
                V x = src[r * nb + (SH && !XL ? (r * nb) >> SH : 0)];
                if (r > 0 && LGNS > 0) x = vmul(x, w[r]);
                v[t][r] = x;
            }
        }
    }
}

// Radix-R DFT of the loaded butterflies and the Stockham store (through policy st).
// XL = 1: the output is stored XOR-swizzled, element i at (i ^ ((i >> 4) & 7)) of a row of 2^LGL
// (Ns = 1 radix-16 passes only).  Their stores write 16 j + r for lane j, which the pad layout
// puts 2-way on the banks of every group of 8 lanes; swizzled, the 8 lanes hit 8 distinct
// 16-B banks, and the next pass's reads (j + r nb, nb a multiple of 128) stay conflict-free.
template <int R, bool INV, int NB, int SH, int NTHR, int LGL, int LGNS, int XL = 0, class V, class St>
__device__ __forceinline__ void sh_store(V (&v)[NB][R], int rs, int nrows, const St& st) {
    constexpr int lgR = clog2(R);
    constexpr int lgnb = LGL - lgR;
    constexpr int nb = 1 << lgnb;
    constexpr int Ns = 1 << LGNS;
    static_assert(!XL || (LGNS == 0 && R == 16), "XOR-swizzled output: Ns = 1 radix-16 passes");
    const int total = nb * nrows;
#pragma unroll
    for (int t = 0; t < NB; ++t) {
        const int beta = threadIdx.x + t * NTHR;
        if (beta < total) {
            const int row = beta >> lgnb, j = beta & (nb - 1);
            const int k = j & (Ns - 1);
            Dft<R, INV, V>::run(v[t]);
            const int idxD = ((j >> LGNS) << (LGNS + lgR)) + k;
            if constexpr (XL) {
                const int wbase = (row << LGL) + idxD, c = j & 7;
#pragma unroll
                for (int r = 0; r < R; ++r) st.put(t * R + r, row, idxD + r, wbase + (r & 8) + ((r & 7) ^ c), v[t][r]);
            } else {
                const int wbase = row * rs + lidx<SH>(idxD);
#pragma unroll
                for (int r = 0; r < R; ++r)
                    st.put(t * R + r, row, idxD + r * Ns, wbase + r * Ns + (SH ? (r * Ns) >> SH : 0), v[t][r]);
            }
        }
    }
}

// TAIL = false: no barrier after the pass (the caller's next LDS writes go to other rows).
template <int R, bool INV, int NB, int SH, int NTHR, int LGL, int LGNS, bool CMP, int XL = 0, bool TAIL = true, class V,
          class TW, class St>
__device__ __forceinline__ void sh_pass(V* buf, int rs, int nrows, const TW& tw, const St& st) {
    V v[NB][R];
    sh_load<R, INV, NB, SH, NTHR, LGL, LGNS, CMP, XL>(buf, rs, nrows, tw, v);
    if constexpr (StoresLds<St>::value) RSP_WAR_SYNC();
    sh_store<R, INV, NB, SH, NTHR, LGL, LGNS>(v, rs, nrows, st);
    if constexpr (TAIL) __syncthreads();
}

// Passes Q..QEND-1 of a 2^LG-point FFT (radix order reversed if REV) over `nrows` rows;
// pass n_passes - 1 stores through `last`, the others through `mid`.  tw = this plan's
// concatenated tables.  PTS = complex points per thread (nrows * L / NTHR).
template <int LG, int Q, int QEND, int LGNS, int PTS, bool INV, bool REV, int SH, int NTHR, bool CMP, bool PAL = false,
          int XIN = 0, bool TAIL = true, class V, class TW, class StMid, class StLast>
__device__ __forceinline__ void fft_range(V* buf, int rs, int nrows, const TW& tw, const StMid& mid, const StLast& last) {
    constexpr int NP = n_passes(LG);
    if constexpr (Q < QEND) {
        constexpr int RB = rad_bits_p(LG, Q, REV, PAL);
        constexpr int R = 1 << RB;
        constexpr int NB = (PTS + R - 1) / R;
        const auto twq = tw + tw_pass_off(LG, Q, REV, CMP, PAL);
        if constexpr (Q == NP - 1)
            sh_pass<R, INV, NB, SH, NTHR, LG, LGNS, CMP, XIN, TAIL>(buf, rs, nrows, twq, last);
        else
            sh_pass<R, INV, NB, SH, NTHR, LG, LGNS, CMP, XIN>(buf, rs, nrows, twq, mid);
        fft_range<LG, Q + 1, QEND, LGNS + RB, PTS, INV, REV, SH, NTHR, CMP, PAL, 0, TAIL>(buf, rs, nrows, tw, mid, last);
    }
}

// All passes of a 2^LG-point FFT over `nrows` rows; the last pass stores through `last`
// (TAIL: followed by a barrier).
template <int LG, int PTS, int SH, int NTHR, bool TAIL = true, class V, class StMid, class StLast>
__device__ __forceinline__ void fft_passes(V* buf, int rs, int nrows, const V* tw, const StMid& mid,
                                           const StLast& last) {
    fft_range<LG, 0, n_passes(LG), 0, PTS, false, false, SH, NTHR, false, false, 0, TAIL>(buf, rs, nrows, tw, mid, last);
}

// ---- Stockham passes of any length L and radix R (mixed-radix overlap-save blocks) ----------
// Same formulation as sh_load / sh_store with L, R, Ns compile-time constants that need not be
// powers of two: divisions by them become multiply-shifts, and every LDS index is padded per
// element (lidx of the full position).
// Padded LDS offset of element j + r D of a row when it splits into a per-thread base lidx(j) plus
// a compile-time offset: always when D is a multiple of the pad period 2^SH ((j + r D) >> SH =
// (j >> SH) + r D / 2^SH); with DIVP also when D divides 2^SH and the thread's j mod 2^SH < D
// (shg_store: idxD = (j / NS) NS R + j mod NS with NS R a multiple of 2^SH), where the carry of
// j mod 2^SH + r D past 2^SH is that of r D alone.
template <int SH, int D, bool DIVP = false>
constexpr bool lidx_sep() {
    return SH == 0 || D % (1 << SH) == 0 || (DIVP && (1 << SH) % D == 0);
}
template <int SH, int D>
constexpr int lidx_off(int r) {
    return r * D + (SH ? (r * D) >> SH : 0);
}

template <int R, bool INV, int NB, int SH, int NTHR, int L, int NS, bool CMP, int XL = 0, class V, class TW>
__device__ __forceinline__ void shg_load(const V* buf, int rs, int nrows, const TW& tw, V (&v)[NB][R],
                                         int tix = threadIdx.x) {
    constexpr int nb = L / R;
    static_assert(!XL || nb % 128 == 0, "XOR-swizzled input needs r nb to keep the swizzle bits");
    constexpr bool SEP = lidx_sep<SH, nb>();
    const int total = nb * nrows;
#pragma unroll
    for (int t = 0; t < NB; ++t) {
        const int beta = tix + t * NTHR;
        if (beta < total) {
            const int row = beta / nb, j = beta - row * nb;
            const V* src = XL ? buf + row * L + (j ^ ((j >> 4) & 7)) : buf + row * rs + (SEP ? lidx<SH>(j) : 0);
            V w[R];
            if (NS > 1) load_tw<R, INV, CMP, NS>(tw + (CMP ? j % NS : (j % NS) * tw_row(R, CMP)), w);
#pragma unroll
            for (int r = 0; r < R; ++r) {
                V x = XL ? src[r * nb] : (SEP ? src[lidx_off<SH, nb>(r)] : src[lidx<SH>(j + r * nb)]);
                if (r > 0 && NS > 1) x = vmul(x, w[r]);
                v[t][r] = x;
            }
        }
    }
}
template <int R, bool INV, int NB, int SH, int NTHR, int L, int NS, int XL = 0, class V, class St>
__device__ __forceinline__ void shg_store(V (&v)[NB][R], int rs, int nrows, const St& st, int tix = threadIdx.x) {
    constexpr int nb = L / R;
    static_assert(!XL || (NS == 1 && R == 16), "XOR-swizzled output: Ns = 1 radix-16 passes");
    const int total = nb * nrows;
#pragma unroll
    for (int t = 0; t < NB; ++t) {
        const int beta = tix + t * NTHR;
        if (beta < total) {
            const int row = beta / nb, j = beta - row * nb;
            Dft<R, INV, V>::run(v[t]);
            const int idxD = (j / NS) * (NS * R) + j % NS;
            if constexpr (XL) {
                const int wbase = row * L + idxD, c = j & 7;
#pragma unroll
                for (int r = 0; r < R; ++r) st.put(t * R + r, row, idxD + r, wbase + (r & 8) + ((r & 7) ^ c), v[t][r]);
            } else if constexpr (lidx_sep<SH, NS, (NS * R) % (1 << SH) == 0>()) {
                const int wbase = row * rs + lidx<SH>(idxD);
#pragma unroll
                for (int r = 0; r < R; ++r) st.put(t * R + r, row, idxD + r * NS, wbase + lidx_off<SH, NS>(r), v[t][r]);
            } else {
#pragma unroll
                for (int r = 0; r < R; ++r)
                    st.put(t * R + r, row, idxD + r * NS, row * rs + lidx<SH>(idxD + r * NS), v[t][r]);
            }
        }
    }
}
template <int R, bool INV, int NB, int SH, int NTHR, int L, int NS, bool CMP, int XL = 0, class V, class TW, class St>
__device__ __forceinline__ void shg_pass(V* buf, int rs, int nrows, const TW& tw, const St& st) {
    V v[NB][R];
    shg_load<R, INV, NB, SH, NTHR, L, NS, CMP, XL>(buf, rs, nrows, tw, v);
    RSP_WAR_SYNC();
    shg_store<R, INV, NB, SH, NTHR, L, NS>(v, rs, nrows, st);
    __syncthreads();
}

__device__ __forceinline__ int ilog2(int x) { return 31 - __clz(x); }

// One dynamic LDS allocation shared by every kernel of this file (each casts it to its types).
extern __shared__ __attribute__((aligned(16))) unsigned char rsp_lds[];

// Compacted used-sample index n' -> fast-time sample (Geometry::ivl_*).  Constant indices
// only: a per-lane index into the kernel-argument arrays would become a vector load, and its
// s_waitcnt vmcnt(0) would wait for every earlier vector memory op (e.g. pending z stores).
__device__ __forceinline__ int used_sample(const Geometry& g, int np) {
    int lo_q = g.ivl_lo[0], st_q = g.ivl_start[0];
#pragma unroll
    for (int i = 1; i < RSP_MAX_IVL; ++i)
        if (i < g.nivl && np >= g.ivl_start[i]) {
            lo_q = g.ivl_lo[i];
            st_q = g.ivl_start[i];
        }
    return lo_q + np - st_q;
}

// z (compacted Doppler-domain rows) addressing: row (b, v), compacted sample n'.
__device__ __forceinline__ size_t zaddr(const Geometry& g, int b, int v, int np) {
    const int lgNZ = ilog2(g.NZ);
    return (((size_t)b * g.nzc + (np >> lgNZ)) * g.P + v) * g.NZ + (np & (g.NZ - 1));
}

// ======================================================================================
// K1: DBF + MTD window + slow-time FFT + fftshift -> compacted rows
// ======================================================================================
#define K1_THREADS 512
#define K1_SH 4   // LDS pad shift of the slow-time FFT rows (row stride P + P/16)

// DBF (fsf:93-97) on the matrix cores as a real GEMM: D[16 rows x 16 pulses] += A[16 x 4
// channels] * B[4 channels x 16 pulses], rows = (Re, Im) x 8 beams of conj(W), one MFMA per
// (channel group, Re/Im part of x).  A lane's 16-B load is its B operand:
//  - float: v_mfma_f32_16x16x4f32; the load holds pulses (p, p+1) of one channel (re, im, re,
//    im), the B operand of two column blocks (even / odd pulses); D row 4*(lane>>4) + i.
//  - double: v_mfma_f64_16x16x4f64; the load holds one pulse (re, im); D row (lane>>4) + 4*i
//    (the f64 C/D layout, cdna_hip_programming.md section 3).
template <class T> struct Dbf;
template <> struct Dbf<float> {
    static constexpr int PPL = 2, NACC = 2;
    typedef f32x4 Ld;
    typedef f32x4 Acc;
    static __device__ __forceinline__ Ld bits(u32x4 t) { return __builtin_bit_cast(f32x4, t); }
    static __device__ __forceinline__ void mma(Acc (&acc)[NACC], float are, float aim, Ld x) {
        acc[0] = __builtin_amdgcn_mfma_f32_16x16x4f32(are, x.x, acc[0], 0, 0, 0);
        acc[0] = __builtin_amdgcn_mfma_f32_16x16x4f32(aim, x.y, acc[0], 0, 0, 0);
        acc[1] = __builtin_amdgcn_mfma_f32_16x16x4f32(are, x.z, acc[1], 0, 0, 0);
        acc[1] = __builtin_amdgcn_mfma_f32_16x16x4f32(aim, x.w, acc[1], 0, 0, 0);
    }
    static __device__ __forceinline__ int row(int grp, int i) { return 4 * grp + i; }
};
template <> struct Dbf<double> {
    static constexpr int PPL = 1, NACC = 1;
    typedef d2 Ld;
    typedef f64x4 Acc;
    static __device__ __forceinline__ Ld bits(u32x4 t) { return __builtin_bit_cast(d2, t); }
    static __device__ __forceinline__ void mma(Acc (&acc)[NACC], double are, double aim, Ld x) {
        acc[0] = __builtin_amdgcn_mfma_f64_16x16x4f64(are, x.x, acc[0], 0, 0, 0);
        acc[0] = __builtin_amdgcn_mfma_f64_16x16x4f64(aim, x.y, acc[0], 0, 0, 0);
    }
    static __device__ __forceinline__ int row(int grp, int i) { return grp + 4 * i; }
};

// D of one sub-tile (sample nl, pulses p .. p + PPL*... of this lane) x window -> padded LDS
// columns [b * NT + nl][Ppad] (Re / Im parts as two scalar stores).
// plim: pulses >= plim (the last sub-tile's lanes past P when P is not a multiple of 16) are not
// stored.
template <class T, int MB>
__device__ __forceinline__ void dbf_store(T* Yf, const typename Dbf<T>::Acc (&acc)[MB][Dbf<T>::NACC], int grp, int B,
                                          int NT, int Ppad, int nl, int p, const T (&w)[Dbf<T>::NACC], int sh,
                                          int plim) {
    if constexpr (sizeof(T) == 8) {
        // double: registers i and i + 2 hold Re and Im of the same beam (rows grp + 4 i and
        // grp + 4 i + 8), so each beam's complex value goes out as one 16-B store.  Two 8-B
        // stores of the parts at a 16-B lane stride put lanes l and l + 8 on the same banks of
        // the 32-bank write path (2-way); the 16-B stores of 8 consecutive lanes cover the 32
        // banks once.
        const int ip = sh ? p + (p >> K1_SH) : p;
#pragma unroll
        for (int mb = 0; mb < MB; ++mb)
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                const int b = mb * 8 + ((grp + 4 * i) & 7);
                if (b < B && p < plim)
                    reinterpret_cast<d2*>(Yf)[(b * NT + nl) * Ppad + ip] =
                        d2{acc[mb][0][i] * w[0], acc[mb][0][i + 2] * w[0]};
            }
        return;
    }
#pragma unroll
    for (int a = 0; a < Dbf<T>::NACC; ++a) {
        const int pa = p + a;
        const int ip = sh ? pa + (pa >> K1_SH) : pa;
#pragma unroll
        for (int mb = 0; mb < MB; ++mb)
#pragma unroll
            for (int i = 0; i < 4; ++i) {   // D row m: beam mb*8 + (m & 7), part m >> 3
                const int m = Dbf<T>::row(grp, i);
                const int b = mb * 8 + (m & 7);
                if (b < B && pa < plim) Yf[2 * ((b * NT + nl) * Ppad + ip) + (m >> 3)] = acc[mb][a][i] * w[a];
            }
    }
}

// Last slow-time FFT pass straight from registers to z with fftshift (fsf:135): column
// row = b NT + nl, frequency o -> Doppler cell v = (o + P/2) mod P.  16 lanes of a butterfly
// group write consecutive v of one column (64 B apart) and the next 16 lanes the neighbouring
// column, so the lines fill within the workgroup.
template <class V>
struct StoreZ {
    __amdgpu_buffer_rsrc_t z; int lgNT, nzc, tile, P, half, lgNZ;
    __device__ __forceinline__ void put(int, int row, int o, int, V x) const {
        const int b = row >> lgNT, nl = row & ((1 << lgNT) - 1);
        const int v = (o + half) & (P - 1);
        const int np = (tile << lgNT) + nl;   // compacted sample
        buf_st<RSP_Z_AUX>(z, (unsigned)(((((b * nzc + (np >> lgNZ)) * P + v) << lgNZ) + (np & ((1 << lgNZ) - 1)))) * (unsigned)sizeof(V), x);
    }
};

// In-place decimation-in-frequency FFT of length P = 16 R1 over nrows LDS rows (stride rs, pads
// per 2^SH), two passes:
//   A: radix 16 over x[n1 R1 + n2] (n1 < 16), output k1 times W_P^(n2 k1), written back to the
//      slots it was read from (n1 -> k1): no thread writes a slot another reads, so the pass
//      needs no read/write barrier (a Stockham pass does);
//   B: radix R1 over the R1 contiguous y[k1 R1 + n2] -> X[k1 + 16 k2], stored through st with
//      the natural bin o = k1 + 16 k2 (the z store applies fftshift).
// twd = the compact pass-A table in LDS, [i][n2] = W_P^(n2 2^i) (load_tw).  Same arithmetic per
// output as the radix-16 x radix-R1 Stockham plan, with the twiddles on the other side.
// PTS = points per thread (nrows P <= PTS NTHR, k1_persistent_fits).
// Which K1 slow-time FFTs run k1_fft_dif (the persistent and the tiled K1 agree, so their outputs
// are bit-identical): P = 64, 128 always; P = 256 for plans of more than 8 channels (with 8, the
// persistent K1's 8 sub-tiles of loads per wave and the DIF's registers spill: the Stockham passes)
__host__ __device__ constexpr bool k1_dif(int lgp, int cp) { return lgp >= 6 && (lgp <= 7 || (lgp == 8 && cp >= 16)); }
#define K1_DIF k1_dif(LGP, CP)

template <int LGP, int PTS, int NTHR, int SH, class V, class St>
__device__ __forceinline__ void k1_fft_dif(V* buf, int rs, int nrows, const V* twd, const St& st) {
    constexpr int P = 1 << LGP, R1 = P / 16, LGR1 = LGP - 4;
    static_assert(R1 >= 4 && R1 <= 16, "P in 64..256");
    {
        const int total = R1 * nrows;
        constexpr int NB = (PTS + 15) / 16;
#pragma unroll
        for (int t = 0; t < NB; ++t) {
            const int beta = threadIdx.x + t * NTHR;
            if (beta < total) {
                const int row = beta >> LGR1, n2 = beta & (R1 - 1);
                V* src = buf + row * rs;
                V x[16];
#pragma unroll
                for (int n1 = 0; n1 < 16; ++n1) x[n1] = src[lidx<SH>(n1 * R1 + n2)];
                V b[4];   // W^(n2 2^i)
#pragma unroll
                for (int i = 0; i < 4; ++i) b[i] = twd[i * R1 + n2];
                Dft<16, false, V>::run(x);
                // W^(n2 k1) for k1 = 1..15 as in load_tw (w[r] = w[2^hb] w[r - 2^hb]), each applied
                // as soon as it exists so that only w[1..8] stay live
                V w[16];
#pragma unroll
                for (int k1 = 1; k1 < 16; ++k1) {
                    const int hb = 1 << clog2(k1);
                    w[k1] = (hb == k1) ? b[clog2(k1)] : vmul(w[hb], w[k1 - hb]);
                    x[k1] = vmul(x[k1], w[k1]);
                }
#pragma unroll
                for (int k1 = 0; k1 < 16; ++k1) src[lidx<SH>(k1 * R1 + n2)] = x[k1];
            }
        }
    }
    __syncthreads();
    {
        const int total = 16 * nrows;
        constexpr int NB = (16 * PTS + P - 1) / P;
#pragma unroll
        for (int t = 0; t < NB; ++t) {
            const int beta = threadIdx.x + t * NTHR;
            if (beta < total) {
                const int row = beta >> 4, k1 = beta & 15;
                const V* src = buf + row * rs;
                V y[R1];
#pragma unroll
                for (int n2 = 0; n2 < R1; ++n2) y[n2] = src[lidx<SH>(k1 * R1 + n2)];
                Dft<R1, false, V>::run(y);
#pragma unroll
                for (int k2 = 0; k2 < R1; ++k2) st.put(k2, row, k1 + 16 * k2, 0, y[k2]);
            }
        }
    }
}

// Slow-time FFT of every (beam, sample) column in LDS for the runtime log2(P); the last pass
// stores through `last`.
template <class V, class StLast>
__device__ __forceinline__ void k1_fft(int lgp, V* Y, int Ppad, int ncols, const V* twl, const StLast& last, bool dif8) {
    StoreLds<V> st{Y};
    switch (lgp) {
        case 4: fft_passes<4, 16, K1_SH, K1_THREADS>(Y, Ppad, ncols, twl, st, last); break;
        case 5: fft_passes<5, 16, K1_SH, K1_THREADS>(Y, Ppad, ncols, twl, st, last); break;
        case 6: k1_fft_dif<6, 16, K1_THREADS, K1_SH>(Y, Ppad, ncols, twl, last); break;   // twl = twD
        case 7: k1_fft_dif<7, 16, K1_THREADS, K1_SH>(Y, Ppad, ncols, twl, last); break;
        case 8:
            if (dif8) k1_fft_dif<8, 16, K1_THREADS, K1_SH>(Y, Ppad, ncols, twl, last);
            else fft_passes<8, 16, K1_SH, K1_THREADS>(Y, Ppad, ncols, twl, st, last);
            break;
        default: fft_passes<9, 16, K1_SH, K1_THREADS>(Y, Ppad, ncols, twl, st, last); break;
    }
}

// ---- factored slow-time DFT for P = R Q (R = 2 or 4, Q odd >= 3; the reference frame's
// P = 332 = 4 x 83, v8:57), decimation in frequency:
//   X[R k1 + k2] = sum_{n1 < Q} W_Q^(n1 k1) y_k2[n1],  y_k2[n1] = W_P^(n1 k2) sum_{n2 < R} x[n1 + Q n2] W_R^(n2 k2)
// Pass 1 (thread per column and n1 <= (Q - 1) / 2): the radix-R DFTs of x[n1 + Q n2] and of its
// mirror x[Q - n1 + Q n2], their twiddles, and the fold of the Q-point stage
//   s_k2[n] = y_k2[n] + y_k2[Q - n] -> slot n + Q k2,   d_k2[n] = y_k2[n] - y_k2[Q - n] -> slot Q - n + Q k2
// in place (a thread writes exactly the slots it read).  Pass 2: with theta = 2 pi k1 n / Q,
//   A = y[0] + sum_{n=1}^{(Q-1)/2} s_n cos(theta),  Bv = sum_n d_n sin(theta),
//   X[R k1 + k2] = A - i Bv,   X[R (Q - k1) + k2] = A + i Bv          (k1 = 0 .. (Q - 1) / 2)
// -- 4 real FMAs per (k1, n) for two outputs, a quarter of the direct sum.  One lane per
// subsequence (column, k2), a wave-uniform set of RQ_RK frequencies per wave: the (cos, sin)
// pair of a step is the same for every lane (an LDS broadcast read), the lane's s_n and d_n two
// 16-B reads shared by its RQ_RK frequencies.  twq = [fset][n - 1][r] (twQ, in LDS), twp =
// W_P^i, i < P (in LDS); st.put(col, o, x) stores output bin o of column col.
template <int R, int NTHR, class V, class St>
__device__ __forceinline__ void k1_dft_rq(V* buf, int rs, int ncols, int Q, const V* twq, const V* twp, const St& st) {
    const int Qh = (Q - 1) >> 1, KH = Qh + 1;
    {   // ---- pass 1
        const int items = ncols * KH;
        for (int it = threadIdx.x; it < items; it += NTHR) {
            const int c = it / KH, n1 = it - c * KH;
            V* col = buf + c * rs;
            V u[R];
#pragma unroll
            for (int n2 = 0; n2 < R; ++n2) u[n2] = col[n1 + Q * n2];
            Dft<R, false, V>::run(u);
            if (n1 == 0) {   // W_P^0 = 1; y[0] is its own mirror
#pragma unroll
                for (int k2 = 0; k2 < R; ++k2) col[Q * k2] = u[k2];
                continue;
            }
            V v[R];
            const int m = Q - n1;
#pragma unroll
            for (int n2 = 0; n2 < R; ++n2) v[n2] = col[m + Q * n2];
            Dft<R, false, V>::run(v);
            col[n1] = u[0] + v[0];
            col[m] = u[0] - v[0];
#pragma unroll
            for (int k2 = 1; k2 < R; ++k2) {   // n1 k2, m k2 < Q R = P: direct table entries
                const V a = vmul(u[k2], twp[n1 * k2]), b = vmul(v[k2], twp[m * k2]);
                col[n1 + Q * k2] = a + b;
                col[m + Q * k2] = a - b;
            }
        }
    }
    __syncthreads();
    {   // ---- pass 2
        const int NS = ncols * R, nfs = (KH + RQ_RK - 1) / RQ_RK, ngrp = (NS + 63) >> 6;
        const int lane = threadIdx.x & 63;
        const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
        for (int item = wv; item < ngrp * nfs; item += NTHR / 64) {   // wave-uniform
            const int grp = item / nfs, fs = item - grp * nfs;
            const int sub = grp * 64 + lane;
            const int sc = min(sub, NS - 1);   // idle lanes read a real column, store nothing
            const int c = sc / R, k2 = sc - c * R;
            const V* col = buf + c * rs + Q * k2;   // s_n = col[n], d_n = col[Q - n]
            const V* tw = twq + fs * Qh * RQ_RK;
            V A[RQ_RK], Bv[RQ_RK];
            const V y0 = col[0];
#pragma unroll
            for (int r = 0; r < RQ_RK; ++r) {
                A[r] = y0;
                Bv[r] = V{};
            }
            // software-pipelined: step n + 1's operands are read while step n computes, so one LDS
            // latency is exposed per step instead of one per (cos, sin) pair.  The reads past the
            // last step (s_(Qh+1), d_Qh, the next table row) stay inside the LDS tile / tables and
            // are never used.  Pointer steps keep every address a base plus an immediate offset.
            // Two register sets alternate: the reads of the step after next go out before this
            // step's FMAs (the scheduling barriers keep that order), so a read has a whole step of
            // FMAs to land.  Steps are taken in pairs; the second step of the last pair exists only
            // when Qh is even (uniform).
            const V* ps = col + 1;
            const V* pd = col + Q - 1;
            const V* pt = tw;
            V s0 = ps[0], d0 = pd[0], t0[RQ_RK];
#pragma unroll
            for (int r = 0; r < RQ_RK; ++r) t0[r] = pt[r];   // (cos, sin): the same address in every lane
            auto fma_step = [&](const V& sv, const V& dv, const V (&tc)[RQ_RK]) {
#pragma unroll
                for (int r = 0; r < RQ_RK; ++r) {
                    A[r] += tc[r].x * sv;
                    Bv[r] += tc[r].y * dv;
                }
            };
            for (int n = 1; n <= Qh; n += 2) {
                const V s1 = ps[1], d1 = pd[-1];
                V t1[RQ_RK];
#pragma unroll
                for (int r = 0; r < RQ_RK; ++r) t1[r] = pt[RQ_RK + r];
                __builtin_amdgcn_sched_barrier(0);
                fma_step(s0, d0, t0);
                __builtin_amdgcn_sched_barrier(0);
                ps += 2;
                pd -= 2;
                pt += 2 * RQ_RK;
                s0 = ps[0];
                d0 = pd[0];
#pragma unroll
                for (int r = 0; r < RQ_RK; ++r) t0[r] = pt[r];
                __builtin_amdgcn_sched_barrier(0);
                if (n + 1 <= Qh) fma_step(s1, d1, t1);
                __builtin_amdgcn_sched_barrier(0);
            }
            if (sub < NS) {
#pragma unroll
                for (int r = 0; r < RQ_RK; ++r) {
                    const int k1 = fs * RQ_RK + r;
                    if (k1 < KH) {
                        st.put(c, R * k1 + k2, V{A[r].x + Bv[r].y, A[r].y - Bv[r].x});   // A - i Bv
                        if (k1 > 0) st.put(c, R * (Q - k1) + k2, V{A[r].x - Bv[r].y, A[r].y + Bv[r].x});
                    }
                }
            }
        }
    }
}

// z store of the factored DFT's outputs: column col = b NT + nl, bin o -> Doppler cell
// v = (o + P/2) mod P (fftshift, fsf:135), compacted sample tile NT + nl.
template <class V>
struct StoreZq {
    __amdgpu_buffer_rsrc_t z; int lgNT, nzc, tile, P, half, lgNZ;
    __device__ __forceinline__ void put(int col, int o, V x) const {
        const int b = col >> lgNT, nl = col & ((1 << lgNT) - 1);
        int v = o + half;
        v = v >= P ? v - P : v;
        const int np = (tile << lgNT) + nl;
        // default cache policy, not non-temporal: one store instruction writes 4 consecutive bins
        // (64 B) of each column and the next one of the wave the other half of the 128-B line,
        // which then merge in L2 (non-temporal partial lines went to HBM unmerged: 1.8x the bytes)
        buf_st<0>(z, (unsigned)((((b * nzc + (np >> lgNZ)) * P + v) << lgNZ) + (np & ((1 << lgNZ) - 1))) *
                         (unsigned)sizeof(V), x);
    }
};

template <class V, class St>
__device__ __forceinline__ void k1_dft_rq_r(int R, V* buf, int rs, int ncols, int Q, const V* twq, const V* twp,
                                            const St& st) {
    if (R == 2) k1_dft_rq<2, K1_THREADS>(buf, rs, ncols, Q, twq, twp, st);
    else k1_dft_rq<4, K1_THREADS>(buf, rs, ncols, Q, twq, twp, st);
}

// BMAX = beams rounded up (4/8/16), CP = channels rounded up (8/16/32).  conj(W) enters as the
// per-lane MFMA A operands (Atab, zero for padded beams/channels), so the DBF has no
// data-dependent branches.  mode 3 = DBF + MTD; mode 0 = transpose only (stage-2 path: the
// input channels are the beams).  Non-power-of-two P = R Q takes the factored DFT (k1_dft_rq),
// any other the direct DFT (O(P^2) per column).
// RQ: the instantiation that runs the factored DFT (its registers stay out of the others).
template <class T, int BMAX, int CP, bool RQ>
__global__ __launch_bounds__(K1_THREADS, 2) void k1_dbf_mtd(Geometry g, DevConsts k, FramePtrs fp, int mode) {
    typedef cx<T> V;
    typedef Dbf<T> D;
    V* Y = reinterpret_cast<V*>(rsp_lds);   // [B][NT][Ppad] | twiddles
    const int f = blockIdx.y, tile = blockIdx.x;
    const int B = g.B, C = g.C, P = g.P, NT = g.NT, Ppad = g.Ppad;
    if (tile == 0 && threadIdx.x == 0 && fp.count[f]) *fp.count[f] = 0;   // K3's detection counter
    V* twl = Y + B * NT * Ppad;
    const bool fft = (mode & 2) && g.pow2P;
    const bool rq = RQ && (mode & 2);   // factored DFT: twl = twQ | W_P^i
    const int sh = fft ? K1_SH : 0;
    // P = 64 .. 256 run the in-place k1_fft_dif (as the persistent K1: the same bits), the other
    // powers of two the Stockham passes
    const bool dif = fft && k1_dif(g.logP, CP);
    const V* __restrict__ twPp = static_cast<const V*>(dif ? k.twD : k.twPp);
    const int ntw = dif ? (P >> 2) : g.twPp_elems;
    const T* __restrict__ win = static_cast<const T*>(k.win);
    // twiddles: global loads issued first, LDS stores after the cube loads are in flight (the
    // barrier before the FFT orders them), so no load waits behind a barrier at kernel start
    constexpr int TWPRE = 2;
    V twv[TWPRE];
#pragma unroll
    for (int u = 0; u < TWPRE; ++u) {
        const int i = threadIdx.x + u * K1_THREADS;
        if (fft && i < ntw) twv[u] = twPp[i];
    }
    const V* __restrict__ x = static_cast<const V*>(fp.in[f]);
    const size_t NP = (size_t)g.cpitch;   // channel stride
    if (mode & 1) {
        constexpr int NJ = CP / 4, MB = BMAX <= 8 ? 1 : 2, TPW = (16 / NJ) / MB > 0 ? (16 / NJ) / MB : 1;
        constexpr int PT = 16 * D::PPL;   // pulses per sub-tile
        const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, grp = lane >> 4, col = lane & 15;
        const T* At = static_cast<const T*>(k.Atab);
        T are[MB][NJ], aim[MB][NJ];   // this lane's A operand: row lane&15, channel 4j + lane>>4
#pragma unroll
        for (int mb = 0; mb < MB; ++mb)
#pragma unroll
            for (int j = 0; j < NJ; ++j) {
                are[mb][j] = At[((mb * NJ + j) * 2 + 0) * 64 + lane];
                aim[mb][j] = At[((mb * NJ + j) * 2 + 1) * 64 + lane];
            }
        const int ptiles = (P + PT - 1) / PT;
        const int ntp = NT * ptiles;
        T* Yf = reinterpret_cast<T*>(Y);
        // a wave takes TPW consecutive sub-tiles (pulse tiles of the same sample first), so the
        // pulse row of each (channel, sample) is fetched by one wave in one burst
        for (int t0 = wv * TPW; t0 < ntp; t0 += (K1_THREADS / 64) * TPW) {
            typename D::Ld xv[TPW][NJ];
            int nlv[TPW], pv[TPW];
#pragma unroll
            for (int u = 0; u < TPW; ++u) {      // every load of TPW sub-tiles in flight together
                const int t = t0 + u;
                const int nl = t / ptiles;
                const int p = (t - nl * ptiles) * PT + D::PPL * col;
                const int np = tile * NT + nl;
                int n = -1;
                if (t < ntp && np < g.nU && p < P) n = used_sample(g, np);
                nlv[u] = t < ntp ? nl : -1;
                pv[u] = p;
#pragma unroll
                for (int j = 0; j < NJ; ++j) {
                    const int c = min(4 * j + grp, C - 1);   // padded channels carry zero weights
                    xv[u][j] = n >= 0 ? D::bits(*reinterpret_cast<const u32x4*>(x + (size_t)c * NP + (size_t)n * P + p))
                                      : typename D::Ld{};
                }
            }
#pragma unroll
            for (int u = 0; u < TPW; ++u) {
                if (nlv[u] < 0) continue;
                typename D::Acc acc[MB][D::NACC];
#pragma unroll
                for (int mb = 0; mb < MB; ++mb) {
#pragma unroll
                    for (int a = 0; a < D::NACC; ++a) acc[mb][a] = typename D::Acc{};
#pragma unroll
                    for (int j = 0; j < NJ; ++j) D::mma(acc[mb], are[mb][j], aim[mb][j], xv[u][j]);
                }
                const int p = pv[u];
                if (p >= P) continue;
                T w[D::NACC];
#pragma unroll
                for (int a = 0; a < D::NACC; ++a) w[a] = (mode & 2) ? win[p + a] : (T)1;
                dbf_store<T, MB>(Yf, acc, grp, B, NT, Ppad, nlv[u], p, w, sh, P);
            }
        }
    } else {
        // ---- transpose only (stage-2 path: input channels are the beams)
        const int items = NT * P;
        for (int it = threadIdx.x; it < items; it += K1_THREADS) {
            const int nl = it / P, p = it - nl * P;
            const int np = tile * NT + nl;
            int n = -1;
            if (np < g.nU) n = used_sample(g, np);
            const int ip = sh ? p + (p >> K1_SH) : p;
#pragma unroll
            for (int b = 0; b < BMAX; ++b) {
                if (b < B) {
                    V val = n >= 0 ? x[(size_t)b * NP + (size_t)n * P + p] : V{};
                    if (mode & 2) val *= win[p];
                    Y[(b * NT + nl) * Ppad + ip] = val;
                }
            }
        }
    }
    if (fft) {
#pragma unroll
        for (int u = 0; u < TWPRE; ++u) {
            const int i = threadIdx.x + u * K1_THREADS;
            if (i < ntw) twl[i] = twv[u];
        }
        for (int i = threadIdx.x + TWPRE * K1_THREADS; i < ntw; i += K1_THREADS) twl[i] = twPp[i];
    }
    if (RQ && rq) {
        const V* __restrict__ twQ = static_cast<const V*>(k.twQ);
        const V* __restrict__ twP = static_cast<const V*>(k.twP);
        for (int i = threadIdx.x; i < g.twq_elems; i += K1_THREADS) twl[i] = twQ[i];
        for (int i = threadIdx.x; i < P; i += K1_THREADS) twl[g.twq_elems + i] = twP[i];
    }
    __syncthreads();
    V* __restrict__ z = static_cast<V*>(fp.z[f]);
    const int zslab = P * NT;   // contiguous [P][NT] slab per (b, tile)
    const int lgNT = ilog2(NT);
    if (!(mode & 2)) {
        for (int e = threadIdx.x; e < B * zslab; e += K1_THREADS) {
            const int b = e / zslab, rem = e - b * zslab;
            const int v = rem >> lgNT, nl = rem & (NT - 1);
            z[zaddr(g, b, v, tile * NT + nl)] = Y[(b * NT + nl) * Ppad + v];
        }
        return;
    }
    const int half = P >> 1;
    if (fft) {
        // ---- P-point FFT of every (b, nl) column (fsf:135); the last pass applies fftshift
        // and stores the [P][NT] slabs from registers
        const StoreZ<V> sz{buf_rsrc(z, (unsigned)(B * g.nzc * P * g.NZ * sizeof(V))), lgNT, g.nzc, tile, P, half, ilog2(g.NZ)};
        k1_fft(g.logP, Y, Ppad, B * NT, twl, sz, k1_dif(8, CP));
    } else if (RQ && rq) {
        const StoreZq<V> sz{buf_rsrc(z, (unsigned)(B * g.nzc * P * g.NZ * sizeof(V))), lgNT, g.nzc, tile, P, half, ilog2(g.NZ)};
        k1_dft_rq_r(g.rqR, Y, Ppad, B * NT, g.rqQ, twl, twl + g.twq_elems, sz);
    } else {
        // non power-of-two P: direct DFT straight to global (O(P^2) per column)
        const V* __restrict__ twP = static_cast<const V*>(k.twP);
        for (int e = threadIdx.x; e < B * zslab; e += K1_THREADS) {
            const int b = e / zslab, rem = e - b * zslab;
            const int v = rem >> lgNT, nl = rem & (NT - 1);
            int kk = v - half;
            if (kk < 0) kk += P;
            const V* colv = Y + (b * NT + nl) * Ppad;
            V acc = V{};
            int idx = 0;
            for (int p = 0; p < P; ++p) {
                acc += vmul(colv[p], twP[idx]);
                idx += kk;
                if (idx >= P) idx -= P;
            }
            z[zaddr(g, b, v, tile * NT + nl)] = acc;
        }
    }
}

// Points per thread of the persistent K1's slow-time FFT (B * NT * P <= K1_PTS * K1_THREADS):
// the plan halves NT for double so that two tile buffers still fit the 160 KB of LDS.
template <class T> constexpr int k1p_pts() { return sizeof(T) == 4 ? 16 : 8; }


// K1, persistent and software-pipelined (the default for power-of-two P when one load round
// covers a tile): one workgroup per CU walks the (frame, tile) list with two LDS tile buffers.
// While tile TT's slow-time FFT runs out of one buffer and its last pass streams z to HBM, the
// cube loads of the workgroup's next tile are already in flight in registers; the DBF of that
// tile then fills the other buffer.  HBM reads and writes overlap instead of alternating
// round by round.  Same arithmetic as k1_dbf_mtd (mode 3).
// TPWX: sub-tiles a wave loads per tile (>= the tiled K1's TPW): 2 TPW when a tile holds more
// sub-tiles than the 8 waves cover at TPW (config #4: 32 channels x 16 beams, NT = 1 sample x
// 256 pulses = 16 sub-tiles, TPW = 1), so that one load round still covers a tile.
template <class T, int BMAX, int CP, int LGP, int TPWX>
__global__ __launch_bounds__(K1_THREADS, 1) void k1p_dbf_mtd(Geometry g, DevConsts k, FramePtrs fp, int nf) {
    typedef cx<T> V;
    typedef Dbf<T> D;
    V* Y = reinterpret_cast<V*>(rsp_lds);   // tile [B][NT][Ppad] x 2 | twiddles
    const int B = g.B, C = g.C, P = g.P, NT = g.NT, Ppad = g.Ppad;
    const int bufsz = B * NT * Ppad;
    V* twl = Y + 2 * bufsz;
    const int total = nf * g.ntiles;
    int TT = blockIdx.x;
    if (TT >= total) return;
    static_assert(LGP >= 6 && LGP <= 8, "the persistent K1 runs P = 64 .. 256 (k1_persistent_fits)");
    if constexpr (K1_DIF) {   // k1_fft_dif's table, 4 x P/16
        const V* __restrict__ twD = static_cast<const V*>(k.twD);
        for (int i = threadIdx.x; i < (P >> 2); i += K1_THREADS) twl[i] = twD[i];
    } else {
        const V* __restrict__ twPp = static_cast<const V*>(k.twPp);
        for (int i = threadIdx.x; i < g.twPp_elems; i += K1_THREADS) twl[i] = twPp[i];
    }
    constexpr int NJ = CP / 4, MB = BMAX <= 8 ? 1 : 2, TPW = TPWX;
    constexpr int PT = 16 * D::PPL;
    const int lane = threadIdx.x & 63, grp = lane >> 4, col = lane & 15;
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);   // wave-uniform: nlv[] and n are scalar
    const T* At = static_cast<const T*>(k.Atab);
    // the conj(W) operands of the MFMA row blocks: held in registers for the kernel's life with
    // one row block (<= 8 beams); with two (16 beams: x4's 32 channels are 64 VGPRs of them) read
    // from LDS (after the twiddles, k1p_lds) in each sub-tile's DBF, which keeps the kernel
    // within 256 VGPRs without scratch
    constexpr bool ALDS = MB == 2;
    T* Al = reinterpret_cast<T*>(twl + P);
    T are[MB][NJ], aim[MB][NJ];
    if constexpr (ALDS) {
        for (int i = threadIdx.x; i < MB * NJ * 2 * 64; i += K1_THREADS) Al[i] = At[i];
    } else {
#pragma unroll
        for (int mb = 0; mb < MB; ++mb)
#pragma unroll
            for (int j = 0; j < NJ; ++j) {
                are[mb][j] = At[((mb * NJ + j) * 2 + 0) * 64 + lane];
                aim[mb][j] = At[((mb * NJ + j) * 2 + 1) * 64 + lane];
            }
    }
    __syncthreads();   // the first DBF reads LDS entries (Atab) other waves wrote
    // this lane's sub-tiles are the same for every tile: (sample nl, pulses p ..) and their
    // window values (k1_persistent_fits guarantees one round: NT * ptiles <= waves * TPWX)
    const int ptiles = P / PT, ntp = NT * ptiles;
    const T* __restrict__ win = static_cast<const T*>(k.win);
    int nlv[TPW], pv[TPW];
    T wv_[TPW][D::NACC];
#pragma unroll
    for (int u = 0; u < TPW; ++u) {
        const int t = wv * TPW + u;
        const int nl = t / ptiles;
        pv[u] = (t - nl * ptiles) * PT + D::PPL * col;
        nlv[u] = t < ntp ? nl : -1;   // pv < P: P >= 64 here; wave-uniform
#pragma unroll
        for (int a = 0; a < D::NACC; ++a) wv_[u][a] = nlv[u] >= 0 ? win[pv[u] + a] : (T)0;
    }
    const size_t NPc = (size_t)g.cpitch;
    // per-lane byte offsets of this lane's (channel, pulses) inside a cube: loop-invariant,
    // so a tile's load issue is scalar sample offsets + buffer loads and writes no VGPR but xv
    // (a VGPR temporary there could be a pending z store's data register: WAR = vmcnt wait)
    unsigned loff[TPW][NJ];
#pragma unroll
    for (int u = 0; u < TPW; ++u)
#pragma unroll
        for (int j = 0; j < NJ; ++j)
            loff[u][j] = (unsigned)(((size_t)min(4 * j + grp, C - 1) * NPc + pv[u]) * sizeof(V));
    const unsigned cube_bytes = (unsigned)((size_t)C * NPc * sizeof(V));
    typename D::Ld xv[TPW][NJ];
    bool vld[TPW];   // wave-uniform: sub-tile u of the tile in flight lies inside the used samples
    auto issue_u = [&](int Tn, int u) {   // cube loads of sub-tile u of tile Tn (fsf:93 operands) into xv[u]
        const int f = __builtin_amdgcn_readfirstlane(Tn / g.ntiles), tile = Tn - f * g.ntiles;
        const __amdgpu_buffer_rsrc_t xr = buf_rsrc(fp.in[f], cube_bytes);
        const int np = tile * NT + nlv[u];
        vld[u] = nlv[u] >= 0 && np < g.nU;
        if (vld[u]) {   // no else: zeroing xv here would wait (vmcnt) on the pending z stores
            const int soff = used_sample(g, np) * P * (int)sizeof(V);
#pragma unroll
            for (int j = 0; j < NJ; ++j)   // non-temporal: the cube is read exactly once
                xv[u][j] = D::bits(__builtin_amdgcn_raw_buffer_load_b128(xr, (int)loff[u][j], soff, 2));
        }
    };
    auto issue = [&](int Tn) {
#pragma unroll
        for (int u = 0; u < TPW; ++u) issue_u(Tn, u);
    };
    // Tnext >= 0 (EARLY2 below): sub-tile u of tile Tnext is loaded into xv[u] as soon as the
    // DBF has read it
    auto dbf = [&](V* buf, int Tnext) {   // MFMA DBF + window of xv into buf (padded rows, K1_SH)
        T* Yf = reinterpret_cast<T*>(buf);
#pragma unroll
        for (int u = 0; u < TPW; ++u) {
            if (nlv[u] < 0) continue;
            typename D::Acc acc[MB][D::NACC];
#pragma unroll
            for (int mb = 0; mb < MB; ++mb)
#pragma unroll
                for (int a = 0; a < D::NACC; ++a) acc[mb][a] = typename D::Acc{};
            if (vld[u]) {   // samples past the used ones: zero columns, like k1_dbf_mtd's n = -1
#pragma unroll
                for (int mb = 0; mb < MB; ++mb)
#pragma unroll
                    for (int j = 0; j < NJ; ++j) {
                        if constexpr (ALDS)
                            D::mma(acc[mb], Al[((mb * NJ + j) * 2 + 0) * 64 + lane], Al[((mb * NJ + j) * 2 + 1) * 64 + lane],
                                   xv[u][j]);
                        else
                            D::mma(acc[mb], are[mb][j], aim[mb][j], xv[u][j]);
                    }
            }
            if (Tnext >= 0) issue_u(Tnext, u);
            dbf_store<T, MB>(Yf, acc, grp, B, NT, Ppad, nlv[u], pv[u], wv_[u], K1_SH, P);
        }
    };
    const int lgNT = ilog2(NT), half = P >> 1;
    // EARLY: the next tile's loads go out as soon as this wave's DBF has read xv, before the tile
    // barrier (x2: K1 -0.6 %, bench +0.6 %; x4, since P = 256 runs the in-place DIF FFT as well:
    // K1 2.13 -> 2.06 ms, profiles/r06zc_k1_p256_dif_ab.txt).  Behind the Stockham passes (P = 256
    // with 8 channels, K1_DIF) the xv registers stay live across them and it cost 36 %.
    constexpr bool EARLY = K1_DIF;
    // EARLY2 (complex single): each sub-tile's loads of the next tile go out inside the DBF, right
    // after the sub-tile's MFMAs have read xv[u] (c64 K1 158-163 -> 151 us; in complex double
    // 226-227 -> 236-238, so double issues after the DBF)
    constexpr bool EARLY2 = EARLY && sizeof(T) == 4;
    issue(TT);
    dbf(Y, EARLY2 && TT + (int)gridDim.x < total ? TT + (int)gridDim.x : -1);
    if (EARLY && !EARLY2 && TT + (int)gridDim.x < total) issue(TT + gridDim.x);
    __syncthreads();
    int cur = 0;
    int it = 0;   // diagnostic builds: the phase stamps' iteration index
    for (; TT < total; TT += gridDim.x, ++it) {
        const int Tn = TT + gridDim.x;
        K1_STAMP(it, 0);
        if (!EARLY && Tn < total) issue(Tn);   // next tile's loads fly during this tile's FFT + z stores
        const int f = __builtin_amdgcn_readfirstlane(TT / g.ntiles), tile = TT - f * g.ntiles;
        if (tile == 0 && threadIdx.x == 0 && fp.count[f]) *fp.count[f] = 0;   // K3's detection counter
        V* __restrict__ z = static_cast<V*>(fp.z[f]);
        const StoreZ<V> sz{buf_rsrc(z, (unsigned)(B * g.nzc * P * g.NZ * sizeof(V))), lgNT, g.nzc, tile, P, half, ilog2(g.NZ)};
        // K1_DIF: in place, one barrier between its two passes (P = 256 as 16 x 16: K1 2.23 -> 2.13
        // ms at x4 against the Stockham passes, which 8-channel plans keep).  No barrier after the
        // last pass: its reads of buffer cur are ordered before the next writes of cur (the next
        // tile's dbf) by the barrier below, and dbf now writes cur ^ 1
        if constexpr (K1_DIF)
            k1_fft_dif<LGP, k1p_pts<T>(), K1_THREADS, K1_SH>(Y + cur * bufsz, Ppad, B * NT, twl, sz);
        else
            fft_passes<LGP, k1p_pts<T>(), K1_SH, K1_THREADS, false>(Y + cur * bufsz, Ppad, B * NT, twl,
                                                                     StoreLds<V>{Y + cur * bufsz}, sz);
        K1_STAMP(it, 1);
        if (Tn < total) {
            dbf(Y + (cur ^ 1) * bufsz, EARLY2 && Tn + (int)gridDim.x < total ? Tn + (int)gridDim.x : -1);
            if (EARLY && !EARLY2 && Tn + (int)gridDim.x < total) issue(Tn + gridDim.x);
        }
        K1_STAMP(it, 2);
        __syncthreads();
        K1_STAMP(it, 3);
        cur ^= 1;
    }
}

// K1 for the factored slow-time DFT (P = R Q, k1_dft_rq; the reference frame's P = 332),
// persistent: one 512-thread workgroup per CU walks the flattened (frame, tile) list of the launch
// with ONE tile buffer -- the tile and the DFT's tables fill the LDS (reference frame: 13 beams x
// 332 pulses x 16 B + 33 KB of tables).  Per tile: the DBF consumes the cube loads already in
// registers, the next tile's loads go out at once (non-temporal), and they land while pass 1 and
// pass 2 run; pass 2 stores z.  Same arithmetic per element as k1_dbf_mtd (mode 3, factored DFT):
// bit-identical outputs.  TPW sub-tiles per wave cover a tile in one load round (k1q_tpw); the
// last sub-tile of a column may run past P (lanes with p >= P load the next row's samples or
// zeros past the cube and store nothing).
template <class T, int BMAX, int CP, int TPW>
__global__ __launch_bounds__(K1_THREADS, 1) void k1q_dbf_mtd(Geometry g, DevConsts k, FramePtrs fp, int nf) {
    typedef cx<T> V;
    typedef Dbf<T> D;
    // LDS: tile [B][NT][Ppad] | twQ | W_P^i | the DBF's MFMA A operands (Atab) -- read from LDS
    // per sub-tile rather than held in registers, which pass 2 needs for its operands in flight
    constexpr int NJ = CP / 4, MB = BMAX <= 8 ? 1 : 2;
    V* Y = reinterpret_cast<V*>(rsp_lds);
    const int B = g.B, C = g.C, P = g.P, NT = g.NT, Ppad = g.Ppad;
    V* twq = Y + B * NT * Ppad;
    V* twp = twq + g.twq_elems;
    T* Al = reinterpret_cast<T*>(twp + P);   // [MB][NJ][Re, Im][64]
    const int total = nf * g.ntiles;
    int TT = blockIdx.x;
    if (TT >= total) return;
    {
        const V* __restrict__ tq = static_cast<const V*>(k.twQ);
        const V* __restrict__ tp = static_cast<const V*>(k.twP);
        const T* __restrict__ At = static_cast<const T*>(k.Atab);
        for (int i = threadIdx.x; i < g.twq_elems; i += K1_THREADS) twq[i] = tq[i];
        for (int i = threadIdx.x; i < P; i += K1_THREADS) twp[i] = tp[i];
        for (int i = threadIdx.x; i < MB * NJ * 2 * 64; i += K1_THREADS) Al[i] = At[i];
    }
    __syncthreads();   // the first DBF reads Atab entries other waves wrote
    constexpr int PT = 16 * D::PPL;
    const int lane = threadIdx.x & 63, grp = lane >> 4, col = lane & 15;
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int ptiles = (P + PT - 1) / PT, ntp = NT * ptiles;
    const T* __restrict__ win = static_cast<const T*>(k.win);
    int nlv[TPW], pv[TPW];
    T wv_[TPW][D::NACC];
#pragma unroll
    for (int u = 0; u < TPW; ++u) {
        // round-robin over the waves: a tile's ntp sub-tiles (21 at the reference frame) split
        // 3/3/3/3/3/2/2/2 rather than 4/4/4/4/4/1, so that the waves sharing a SIMD (w, w + 4)
        // carry 6 + 5 + 5 + 5 of the MFMA work instead of 8 + 5 + 4 + 4
        const int t = u * (K1_THREADS / 64) + wv;
        const int nl = t / ptiles;
        pv[u] = (t - nl * ptiles) * PT + D::PPL * col;
        nlv[u] = t < ntp ? nl : -1;   // wave-uniform
#pragma unroll
        for (int a = 0; a < D::NACC; ++a) wv_[u][a] = (nlv[u] >= 0 && pv[u] + a < P) ? win[pv[u] + a] : (T)0;
    }
    const unsigned NPc = (unsigned)g.cpitch;
    const unsigned cube_bytes = (unsigned)((size_t)C * g.cpitch * sizeof(V));
    typename D::Ld xv[TPW][NJ];
    bool vld[TPW];
    auto issue = [&](int Tn) {   // cube loads of tile Tn (fsf:93 operands) into xv
        const int f = __builtin_amdgcn_readfirstlane(Tn / g.ntiles), tile = Tn - f * g.ntiles;
        const __amdgpu_buffer_rsrc_t xr = buf_rsrc(fp.in[f], cube_bytes);
        int gq = grp;
        asm volatile("" : "+v"(gq));   // the lane offsets are formed here, not kept live across the DFT
#pragma unroll
        for (int u = 0; u < TPW; ++u) {
            const int np = tile * NT + nlv[u];
            vld[u] = nlv[u] >= 0 && np < g.nU;
            if (vld[u]) {
                const int soff = used_sample(g, np) * P * (int)sizeof(V);
#pragma unroll
                for (int j = 0; j < NJ; ++j) {   // non-temporal: the cube is read exactly once
                    const unsigned lo = ((unsigned)min(4 * j + gq, C - 1) * NPc + (unsigned)pv[u]) * (unsigned)sizeof(V);
                    xv[u][j] = D::bits(__builtin_amdgcn_raw_buffer_load_b128(xr, (int)lo, soff, 2));
                }
            }
        }
    };
    const int lgNT = ilog2(NT), half = P >> 1;
    issue(TT);
    int it = 0;   // diagnostic builds: the phase stamps' iteration index
    for (; TT < total; TT += gridDim.x, ++it) {
        const int Tn = TT + gridDim.x;
        K1_STAMP(it, 0);
        {   // MFMA DBF + window of xv into Y
            T* Yf = reinterpret_cast<T*>(Y);
#pragma unroll
            for (int u = 0; u < TPW; ++u) {
                if (nlv[u] < 0) continue;
                typename D::Acc acc[MB][D::NACC];
#pragma unroll
                for (int mb = 0; mb < MB; ++mb)
#pragma unroll
                    for (int a = 0; a < D::NACC; ++a) acc[mb][a] = typename D::Acc{};
                if (vld[u]) {   // samples past the used ones: zero columns
#pragma unroll
                    for (int mb = 0; mb < MB; ++mb)
#pragma unroll
                        for (int j = 0; j < NJ; ++j)
                            D::mma(acc[mb], Al[((mb * NJ + j) * 2 + 0) * 64 + lane], Al[((mb * NJ + j) * 2 + 1) * 64 + lane],
                                   xv[u][j]);
                }
                dbf_store<T, MB>(Yf, acc, grp, B, NT, Ppad, nlv[u], pv[u], wv_[u], 0, P);
            }
        }
        if (Tn < total) issue(Tn);   // the next tile's loads fly during this tile's DFT
        K1_STAMP(it, 1);
        const int f = __builtin_amdgcn_readfirstlane(TT / g.ntiles), tile = TT - f * g.ntiles;
        if (tile == 0 && threadIdx.x == 0 && fp.count[f]) *fp.count[f] = 0;   // K3's detection counter
        __syncthreads();   // the tile (and, the first time, the tables) in LDS
        K1_STAMP(it, 2);
        V* __restrict__ z = static_cast<V*>(fp.z[f]);
        const StoreZq<V> sz{buf_rsrc(z, (unsigned)(B * g.nzc * P * g.NZ * sizeof(V))), lgNT, g.nzc, tile, P, half, ilog2(g.NZ)};
        k1_dft_rq_r(g.rqR, Y, Ppad, B * NT, g.rqQ, twq, twp, sz);
        K1_STAMP(it, 3);
        __syncthreads();   // pass 2's reads of Y before the next DBF writes it
    }
}

// ======================================================================================
// K2: pulse compression of every row (fsf:101-126)
// ======================================================================================
template <class V>
struct StoreRdm {   // last inverse pass: keep outputs i in [Lh-1, Lh-1+V) that map to gates < gend;
                    // also writes |x| (the CFAR input, fsf:184-185) into the magnitude map.
                    // Branch-free: rejected outputs get an out-of-range buffer offset.
    __amdgpu_buffer_rsrc_t rdm, mag; int G; int Gp; int row0; int rows_total; int Lh1; int g0; int gend; bool has_rdm;
    __device__ __forceinline__ void put(int, int row, int o, int, V x) const {
        const int gg = g0 + o - Lh1;
        const int rho = row0 + row;
        const bool ok = o >= Lh1 && gg < gend && rho < rows_total;
        if (has_rdm) buf_st<RSP_RDM_AUX>(rdm, ok ? (unsigned)(rho * G + gg) * (unsigned)sizeof(V) : RSP_OOB, x);
        buf_st1(mag, ok ? (unsigned)(rho * Gp + gg) * (unsigned)sizeof(scal<V>) : RSP_OOB, cmag(x));
    }
};
// The same for a pass whose output rows are uniform per wave (or per workgroup): the row's
// resources are built once, before the pass, by the caller; RDM (compile-time) says whether the
// complex map is stored.  The pass is the overlap-save block's last inverse pass with nb = NS
// butterflies per row: thread j's output r is o = j + r NS, so the outputs r < rskip =
// floor(Lh1 / NS) lie below Lh1 -- discarded overlap-save outputs -- for every thread, and their
// |x| and stores are skipped (a uniform branch; only checked for r < R / 2, where they can be).
template <class V, bool RDM, int NS, int R>
struct StoreRowK {
    typedef scal<V> S;
    __amdgpu_buffer_rsrc_t rr, mr;
    unsigned lh1v, lh1s;   // Lh1 in bytes of V / of S
    int rskip;
    __device__ __forceinline__ StoreRowK(V* rdm, S* mag, int G, int Gp, int rho, int rows_total, int Lh1, int g0,
                                         int gend) {
        const unsigned n = rho < rows_total ? (unsigned)(gend - g0) : 0u;
        if (RDM) rr = buf_rsrc(rdm + (size_t)rho * G + g0, n * (unsigned)sizeof(V));
        mr = buf_rsrc(mag + (size_t)rho * Gp + g0, n * (unsigned)sizeof(S));
        lh1v = (unsigned)Lh1 * (unsigned)sizeof(V);
        lh1s = (unsigned)Lh1 * (unsigned)sizeof(S);
        rskip = Lh1 / NS;
    }
    __device__ __forceinline__ void put(int idx, int, int o, int, V x) const {
        const int r = idx % R;
        if (r < R / 2 && r < rskip) return;
        // The masked outputs rely on the wrapped offset being past num_records.  Left visible,
        // (o - Lh1) size = j size - Lh1 size + r NS size is split by the compiler into a wrapped
        // VGPR offset plus an immediate r NS size, and the range check of that sum is not the
        // modular one: the first kept gate of a block was dropped (complex single, maps without
        // the RDM).  The opaque offset keeps the whole (wrapped) value in the VGPR.
        unsigned ov = (unsigned)o * (unsigned)sizeof(V) - lh1v, os = (unsigned)o * (unsigned)sizeof(S) - lh1s;
        asm volatile("" : "+v"(ov), "+v"(os));
        if (RDM) buf_st<RSP_RDM_AUX>(rr, ov, x);
        buf_st1(mr, os, cmag(x));
    }
};

// Samples [lo, hi] of row (b, v) of one segment as one buffer window: z's element index is
// increasing in the compacted sample n' (tile-major, slot-minor), so a resource based at
// n' = off (sample lo) that spans n' = off + hi - lo masks every sample outside [lo, hi] --
// below wraps past num_records, above is past it.  rel(n') = the byte offset of n' in the
// window (may wrap); zrow_window() returns the resource (num_records 0 for rows past
// rows_total, which are uniform per wave here).
struct ZWin {
    __amdgpu_buffer_rsrc_t r;
    int e_lo, PNT, lgNT, NT1;
    __device__ __forceinline__ int rel(int np) const { return (np >> lgNT) * PNT + (np & NT1) - e_lo; }
};
template <class V>
__device__ __forceinline__ ZWin zrow_window(const Geometry& g, const V* z, int rho, int rows_total, int off, int lo,
                                            int hi) {
    ZWin w;
    const int b = rho / g.P, v = rho - b * g.P;
    w.lgNT = ilog2(g.NZ);
    w.NT1 = g.NZ - 1;
    w.PNT = g.P * g.NZ;
    const int nph = off + hi - lo;
    w.e_lo = (off >> w.lgNT) * w.PNT + (off & w.NT1);
    const int e_hi = (nph >> w.lgNT) * w.PNT + (nph & w.NT1);
    const V* base = z + ((size_t)b * g.nzc * g.P + v) * g.NZ + w.e_lo;
    w.r = buf_rsrc(base, rho < rows_total ? (unsigned)(e_hi - w.e_lo + 1) * (unsigned)sizeof(V) : 0u);
    return w;
}

// LDS pad of the overlap-save rows: one complex per 32.  For 16-B elements this keeps every
// ds_read_b128 of a pass conflict-free (a pad per 16 would shift lanes 20-27 of a lane group
// onto lane 12's bank), and the stride-16 stores of the two radix-16 Ns = 1 passes 2-way
// (tools/ab/lds_conflicts64.py)
template <class T> constexpr int k2_sh() { return 5; }
// The 2560-point-sized workgroups (k2_pc<double, 4>): rows without pads and twiddles read from
// L1/L2, so that a workgroup's LDS is the 2560 complex doubles of its row alone (40 KB) and 4 fit a
// CU; SH = 30 makes every pad expression zero.  Measured against 3 per CU with pads and staged
// twiddles: k2_pc -3 % at x2 (profiles/r06zf_k2_w4_ab.txt)
constexpr int K2_NOPAD_SH = 30;
template <class T, bool NOPAD> constexpr int k2_sh_np() { return NOPAD ? K2_NOPAD_SH : k2_sh<T>(); }
// LDS complex slots of a workgroup's rows: pts points (Geometry::k2_pts) + their pads
__host__ __device__ constexpr int k2_lds_data(int pts, int sh) { return pts + (pts >> sh); }

// The block's twiddle tables are staged in LDS next to the rows: a pass's twiddles then arrive
// with its LDS data reads instead of after an L2 round trip (-6% for k2_pc in complex double).
// When the radix plan is a palindrome the inverse plan's table equals the forward one (the
// conjugation happens in load_tw), so one copy serves both.
constexpr bool k2_tw_sym(int LGM) {
    for (int q = 0; q < n_passes(LGM); ++q)
        if (rad_bits_p(LGM, q, false, true) != rad_bits_p(LGM, n_passes(LGM) - 1 - q, false, true))
            return false;
    return true;
}
constexpr int k2_tw_lds(int LGM) {
    return tw_total(LGM, false, true, true) +
           (k2_tw_sym(LGM) ? 0 : tw_total(LGM, true, true, true));
}
constexpr int k2_tw_lds_max() {
    int m = 16 * tw_row(10, true) + 160 * tw_row(16, true);   // k2_fft_job_mix<2560>
    for (int lg = 6; lg <= 11; ++lg) m = k2_tw_lds(lg) > m ? k2_tw_lds(lg) : m;
    return m;
}

// The kept overlap-save outputs of `rows` rows from LDS (in natural order after the inverse FFT's
// last pass) to the maps: output o = Lh1 + e is stitched gate g0 + e (fsf:123-126); |x| into the
// magnitude map (the CFAR input, fsf:184-185) and, when the frame's RD map is requested, x into
// it.  Consecutive lanes take consecutive gates (coalesced, conflict-free LDS reads), and the
// square roots run a few at a time instead of 16 per thread at once at the end of the last pass:
// that pass was k2_pc's register peak (188 VGPRs; with this epilogue 3 workgroups fit per CU).
template <class T, int SH>
__device__ __forceinline__ void k2_epilogue(const cx<T>* L, int rs, int rows, int row0, int rows_total, int Lh1, int g0,
                                            int gend, cx<T>* __restrict__ rdm, T* __restrict__ mag, int G, int Gp) {
    typedef cx<T> V;
    const int nkeep = gend - g0;
    for (int r = 0; r < rows; ++r) {
        const int rho = row0 + r;   // uniform
        if (rho >= rows_total) break;
        const V* src = L + r * rs + Lh1;
        const int pad0 = SH ? Lh1 : 0;
        const __amdgpu_buffer_rsrc_t mr = buf_rsrc(mag + (size_t)rho * Gp + g0, (unsigned)nkeep * (unsigned)sizeof(T));
        if (rdm) {
            const __amdgpu_buffer_rsrc_t rr = buf_rsrc(rdm + (size_t)rho * G + g0, (unsigned)nkeep * (unsigned)sizeof(V));
            for (int e = threadIdx.x; e < nkeep; e += K2_THREADS) {
                const V x = src[e + (SH ? ((pad0 + e) >> SH) : 0)];
                buf_st<RSP_RDM_AUX>(rr, (unsigned)e * (unsigned)sizeof(V), x);
                buf_st1(mr, (unsigned)e * (unsigned)sizeof(T), cmag(x));
            }
        } else {
            for (int e = threadIdx.x; e < nkeep; e += K2_THREADS)
                buf_st1(mr, (unsigned)e * (unsigned)sizeof(T), cmag(src[e + (SH ? ((pad0 + e) >> SH) : 0)]));
        }
    }
}

// x[r] *= H[j + r S] (the filter spectrum, 1/M folded in) for the fused pass's R outputs, loaded
// after the forward DFT that produces them: H then occupies registers only from here to the
// product (an empty asm keeps the loads below the DFT; loaded with the samples it held 64 VGPRs
// of complex double through the whole forward FFT)
template <int R, int S, class V>
__device__ __forceinline__ void k2_apply_h(V (&x)[R], __amdgpu_buffer_rsrc_t hr, int j) {
    asm volatile("" ::: "memory");
    V h[R];
#pragma unroll
    for (int r = 0; r < R; ++r) h[r] = buf_ld<V>(hr, (unsigned)(j + r * S) * (unsigned)sizeof(V));
#pragma unroll
    for (int r = 0; r < R; ++r) x[r] = vmul(x[r], h[r]);
}

// One overlap-save block of one FFT segment for PTS / 2^LGM adjacent rows (PTS = 4096, or 2048
// in a plan whose workgroups are sized for the 2560-point block, Geometry::k2_pts).
// LDS round trips: forward pass 0 runs on the samples as loaded from z; the forward FFT's
// last pass, the filter-spectrum product and the inverse FFT's first pass (radices in
// reverse order, so that pass has the same butterflies) run in registers back to back;
// the inverse FFT's last pass stores the kept gates to HBM.  2 (log2 M / 4) round trips
// instead of 2 (log2 M / 4) + 3.  Twiddles are compact rows, staged in LDS.
// The twiddle source of a K2 job: the LDS copy, or the plan's table in global memory through a
// buffer resource (TwG; x4 k2_pc 2.355 -> 2.347 ms against 64-bit addresses, r06zg)
template <bool LDS, class V>
__device__ __forceinline__ auto k2_tw_src(const V* lds, const V* glob) {
    if constexpr (LDS)
        return lds;
    else
        return TwG<V>{buf_rsrc(glob, RSP_OOB), 0u};
}
template <class T, int LGM, int PTS, bool EPI, bool NOPAD>
__device__ __forceinline__ void k2_fft_job(const Geometry& g, const DevConsts& k, const SegDesc& sd, const K2Job& job,
                                           const cx<T>* __restrict__ z, cx<T>* __restrict__ rdm, T* __restrict__ mag,
                                           int row0, int rows_total, cx<T>* L) {
    typedef cx<T> V;
    constexpr int SH = k2_sh_np<T, NOPAD>();
    constexpr int M = 1 << LGM;
    constexpr int rows = PTS / M > 0 ? PTS / M : 1;
    constexpr int rs = M + (M >> SH);
    constexpr int NP = n_passes(LGM);
    static_assert(NP >= 2, "overlap-save block needs >= 2 FFT passes");
    constexpr bool PAL = true, CMP = true;
    constexpr int RB0 = rad_bits_p(LGM, 0, false, PAL), R0 = 1 << RB0, NB0 = 16 / R0, nb0 = M / R0;
    constexpr int RBL = rad_bits_p(LGM, NP - 1, false, PAL), RL = 1 << RBL, NBL = 16 / RL;   // last forward pass
    const int P = g.P, G = g.G;
    const int lo = sd.lo, hi = sd.hi, off = sd.off;
    const int tid = threadIdx.x;
    const int Lh1 = sd.Lh - 1;
    const int g0 = sd.ga + job.blk * sd.V;
    const int a = sd.seg_lo + g0 - Lh1;           // sample index of u[0]
    const V* twl = static_cast<const V*>(k.twM) + sd.tw_off;
    const V* __restrict__ H = static_cast<const V*>(k.H);
    // every global load of the workgroup in flight together: the 16 samples of this thread's
    // pass-0 butterflies and its 16 filter-spectrum values (for the fused middle pass)
    V v0[NB0][R0];
    const int lgNT = ilog2(g.NZ);
    // one row per wave (nb0 a multiple of 64, one butterfly per thread): the row's sample window
    // is a scalar buffer resource, and a load's offset needs no mask
    constexpr bool WROW = nb0 >= 64 && NB0 == 1;
    if constexpr (WROW) {
        const int rl = __builtin_amdgcn_readfirstlane(tid / nb0);
        // waves past the block's rows (fewer rows than 256 / nb0) load nothing
        const ZWin zw = zrow_window(g, z, row0 + rl, rl < rows ? rows_total : 0, off, lo, hi);
        const int j = tid & (nb0 - 1);
        const int np0 = a + j - lo + off;
        if ((nb0 & (g.NZ - 1)) == 0) {   // uniform: element r sits r (nb0 P) past element 0
            const unsigned e0 = (unsigned)zw.rel(np0) * (unsigned)sizeof(V), st = (unsigned)(nb0 * P) * (unsigned)sizeof(V);
#pragma unroll
            for (int r = 0; r < R0; ++r) v0[0][r] = buf_ld<V>(zw.r, e0 + r * st);
        } else {
#pragma unroll
            for (int r = 0; r < R0; ++r) v0[0][r] = buf_ld<V>(zw.r, (unsigned)zw.rel(np0 + r * nb0) * (unsigned)sizeof(V));
        }
    }
    const __amdgpu_buffer_rsrc_t zr = buf_rsrc(z, (unsigned)(g.B * g.nzc * P * g.NZ * sizeof(V)));
#pragma unroll
    for (int t = 0; t < (WROW ? 0 : NB0); ++t) {
        const int beta = tid + t * K2_THREADS;
        const int rl = beta / nb0, j = beta & (nb0 - 1);
        const int rho = row0 + rl;
        const int b = rho / P, v = rho - b * P;
        // z index of sample n0 + r nb0: when NT | nb0 the tile advances by nb0/NT per r and the
        // in-tile slot is fixed, so element r sits at zb + r (nb0 P) (one multiply per thread)
        const int np0 = a + j - lo + off;
        const int zb = ((b * g.nzc + (np0 >> lgNT)) * P + v) * g.NZ + (np0 & (g.NZ - 1));
        // branch-free: every lane loads (an out-of-range offset when masked)
        if ((nb0 & (g.NZ - 1)) == 0) {   // uniform
#pragma unroll
            for (int r = 0; r < R0; ++r) {
                const int n = a + j + r * nb0;
                const bool ok = rho < rows_total && n >= lo && n <= hi;
                v0[t][r] = buf_ld<V>(zr, ok ? (unsigned)(zb + r * nb0 * P) * (unsigned)sizeof(V) : RSP_OOB);
            }
        } else {
#pragma unroll
            for (int r = 0; r < R0; ++r) {
                const int n = a + j + r * nb0;
                const bool ok = rho < rows_total && n >= lo && n <= hi;
                v0[t][r] = buf_ld<V>(zr, ok ? (unsigned)zaddr(g, b, v, n - lo + off) * (unsigned)sizeof(V) : RSP_OOB);
            }
        }
    }
    const __amdgpu_buffer_rsrc_t hr = buf_rsrc(H + sd.H_off, (unsigned)(M * sizeof(V)));
    // !EPI: H for the last forward pass's outputs j + r M/RL loaded with the samples; butterflies t
    // and t + (M/RL)/NTHR of a thread have the same j (different rows), so only the distinct ones
    constexpr int NHT = !EPI ? ((M / RL) / K2_THREADS >= NBL ? NBL : ((M / RL) / K2_THREADS > 0 ? (M / RL) / K2_THREADS : 1)) : 1;
    V hreg[NHT * RL];
    if constexpr (!EPI) {
#pragma unroll
        for (int t = 0; t < NHT; ++t) {
            const int j = (tid + t * K2_THREADS) & (M / RL - 1);   // last pass: Ns = nb = M / RL, idxD = j
#pragma unroll
            for (int r = 0; r < RL; ++r) hreg[t * RL + r] = buf_ld<V>(hr, (unsigned)(j + r * (M / RL)) * (unsigned)sizeof(V));
        }
    }
    constexpr int NTWF = tw_total(LGM, false, CMP, PAL);
    // twiddles staged in LDS next to the rows; a 4096-point block's (1 088 entries) do not fit the
    // 2-per-CU workgroup's LDS and are read from L1/L2 instead
    constexpr bool TW_LDS = LGM <= 11 && !NOPAD;
    V* twL = L + k2_lds_data(g.k2_pts, SH);
    if constexpr (TW_LDS)
        for (int e = tid; e < k2_tw_lds(LGM); e += K2_THREADS) twL[e] = twl[e];   // visible after the pass-0 barrier
    const auto twF = k2_tw_src<TW_LDS, V>(twL, twl);
    const auto twI = k2_tw_sym(LGM) ? twF : twF + NTWF;
    // forward pass 0 (Ns = 1, no twiddles) straight from the loaded samples
    // the Ns = 1 passes' outputs XOR-swizzled (sh_store) when a middle pass reads them (3 passes)
    constexpr int XZ = (NP == 3 && R0 == 16 && RL == 16 && 1) ? 1 : 0;
    sh_store<R0, false, NB0, SH, K2_THREADS, LGM, 0, XZ>(v0, rs, rows, StoreLds<V>{L});
    __syncthreads();
    K2_STAMP(1);
    // forward passes 1 .. NP-2
    fft_range<LGM, 1, NP - 1, RB0, 16, false, false, SH, K2_THREADS, CMP, PAL, XZ>(L, rs, rows, twF, StoreLds<V>{L},
                                                                               StoreLds<V>{L});
    // fused: forward last pass, x H (1/M folded in), inverse pass 0 of the reversed plan
    {
        V v[NBL][RL];
        sh_load<RL, false, NBL, SH, K2_THREADS, LGM, LGM - RBL, CMP>(L, rs, rows,
                                                                      twF + tw_pass_off(LGM, NP - 1, false, CMP, PAL), v);
        RSP_WAR_SYNC();
#pragma unroll
        for (int t = 0; t < NBL; ++t) {
            Dft<RL, false, V>::run(v[t]);
            // last forward pass: Ns = nb = M / RL, thread j's outputs j + r M / RL
            if constexpr (EPI) {
                k2_apply_h<RL, M / RL>(v[t], hr, (tid + t * K2_THREADS) & (M / RL - 1));
            } else {
#pragma unroll
                for (int r = 0; r < RL; ++r) v[t][r] = vmul(v[t][r], hreg[(t % NHT) * RL + r]);
            }
        }
        sh_store<RL, true, NBL, SH, K2_THREADS, LGM, 0, XZ>(v, rs, rows, StoreLds<V>{L});
        __syncthreads();
    }
    K2_STAMP(3);
    const int gend = min(sd.gb, g0 + sd.V);
    if constexpr (EPI) {
        // inverse passes 1 .. NP-1 (reversed radices) into LDS; then the valid overlap-save outputs
        // = stitched gates go to the maps
        fft_range<LGM, 1, NP, RBL, 16, true, true, SH, K2_THREADS, CMP, PAL, XZ>(L, rs, rows, twI, StoreLds<V>{L},
                                                                               StoreLds<V>{L});
        k2_epilogue<T, SH>(L, rs, rows, row0, rows_total, Lh1, g0, gend, rdm, mag, G, g.Gp);
    } else if constexpr (WROW) {
        // inverse passes 1 .. NP-2 into LDS, then the last one (Ns = nb0, input not swizzled:
        // XZ applies to the pass after an Ns = 1 pass only) stores the kept gates straight into
        // this wave's row of the maps
        fft_range<LGM, 1, NP - 1, RBL, 16, true, true, SH, K2_THREADS, CMP, PAL, XZ>(L, rs, rows, twI, StoreLds<V>{L},
                                                                                   StoreLds<V>{L});
        constexpr int LGNSL = LGM - RB0;
        static_assert(NP >= 3 || XZ == 0, "last pass input is never swizzled");
        const auto twl_last = twI + tw_pass_off(LGM, NP - 1, true, CMP, PAL);
        const int rho = row0 + __builtin_amdgcn_readfirstlane(tid / nb0);
        if (rdm)
            sh_pass<R0, true, NB0, SH, K2_THREADS, LGM, LGNSL, CMP, 0, false>(
                L, rs, rows, twl_last, StoreRowK<V, true, nb0, R0>(rdm, mag, G, g.Gp, rho, rows_total, Lh1, g0, gend));
        else
            sh_pass<R0, true, NB0, SH, K2_THREADS, LGM, LGNSL, CMP, 0, false>(
                L, rs, rows, twl_last, StoreRowK<V, false, nb0, R0>(rdm, mag, G, g.Gp, rho, rows_total, Lh1, g0, gend));
    } else {
        fft_range<LGM, 1, NP, RBL, 16, true, true, SH, K2_THREADS, CMP, PAL, XZ, false>(
            L, rs, rows, twI, StoreLds<V>{L},
            StoreRdm<V>{buf_rsrc(rdm, (unsigned)(rows_total * G * sizeof(V))),
                        buf_rsrc(mag, (unsigned)(rows_total * g.Gp * sizeof(T))), G, g.Gp, row0, rows_total, Lh1, g0,
                        gend, rdm != nullptr});
    }
}

// Mixed-radix overlap-save block M = R0 x R1 x R0, a palindrome: the inverse FFT runs the same
// radices, the fused middle pass (forward last pass, x H, inverse pass 0) has the same
// butterflies on both sides as in k2_fft_job, and the inverse twiddle table equals the forward
// one (conjugated in load_tw).  Two plans:
//  - 2560 = 16 x 10 x 16: one block covers x2's long segment (Lh = 700, 1860 gates), which takes
//    two 2048-point blocks in powers of two -- 37.5% fewer points.  One row per workgroup: the
//    radix-16 passes run 160 butterflies (waves 0-2, the fourth wave skips them), the radix-10
//    passes 256.
//  - 1024 = 8 x 16 x 8 in workgroups sized for 2048 points (the 3-per-CU plans): two rows, and
//    the three Ns = 1 / fused / last passes run 2 x 128 radix-8 butterflies on all 256 threads;
//    as 16 x 4 x 16 those passes ran 2 x 64 radix-16 butterflies on half of them.
template <class T, int M, int R0, int R1, bool EPI, bool NOPAD>
__device__ __forceinline__ void k2_fft_job_mix(const Geometry& g, const DevConsts& k, const SegDesc& sd, const K2Job& job,
                                               const cx<T>* __restrict__ z, cx<T>* __restrict__ rdm, T* __restrict__ mag,
                                               int row0, int rows_total, cx<T>* L) {
    typedef cx<T> V;
    constexpr int SH = k2_sh_np<T, NOPAD>();
    static_assert(M == R0 * R1 * R0, "palindromic 3-pass plan");
    constexpr int rows = M >= 2048 ? 1 : 2048 / M;
    constexpr int rs = M + (M >> SH);
    constexpr bool CMP = true;
    constexpr int nb0 = M / R0;                                          // radix-R0 butterflies per row
    constexpr int NB0 = (nb0 * rows + K2_THREADS - 1) / K2_THREADS;
    constexpr int NB1 = ((M / R1) * rows + K2_THREADS - 1) / K2_THREADS;
    constexpr int NS1 = R0, NS2 = R0 * R1;                               // Ns of passes 1 and 2
    constexpr int TW2 = NS1 * tw_row(R1, CMP);                           // offset of pass 2's table
    constexpr int NTWF = TW2 + NS2 * tw_row(R0, CMP);
    const int P = g.P, G = g.G;
    const int lo = sd.lo, hi = sd.hi, off = sd.off;
    const int tid = threadIdx.x;
    const int Lh1 = sd.Lh - 1;
    const int g0 = sd.ga + job.blk * sd.V;
    const int a = sd.seg_lo + g0 - Lh1;
    const V* twl = static_cast<const V*>(k.twM) + sd.tw_off;
    const V* __restrict__ H = static_cast<const V*>(k.H);
    static_assert(NB0 == 1, "one radix-R0 butterfly per thread");
    static_assert(rows == 1 || nb0 % 64 == 0, "a row per whole wave (its z window is a scalar resource)");
    static_assert(!NOPAD || rows * rs <= 2560, "the row alone fills the 4-per-CU workgroup's LDS");
    static_assert(NOPAD || rows * rs + NTWF <= k2_lds_data(RSP_K2_POINTS, SH) + k2_tw_lds_max(), "fits the 2-per-CU LDS");
    V v0[NB0][R0];
    V hreg[EPI ? 1 : NB0][R0];   // !EPI: the fused pass's H, loaded with the samples
    // threads past the rows' butterflies (waves past them) skip the loads; a row's samples are one
    // scalar buffer window (zrow_window), so the loads need no masks
    const int rl = rows == 1 ? 0 : __builtin_amdgcn_readfirstlane(tid / nb0);
    const int j = tid - rl * nb0;
    if (tid < nb0 * rows) {
        const ZWin zw = zrow_window(g, z, row0 + rl, rows_total, off, lo, hi);
        const int np0 = a + j - lo + off;
        if ((nb0 & (g.NZ - 1)) == 0) {   // uniform
            const unsigned e0 = (unsigned)zw.rel(np0) * (unsigned)sizeof(V), st = (unsigned)(nb0 * P) * (unsigned)sizeof(V);
#pragma unroll
            for (int r = 0; r < R0; ++r) v0[0][r] = buf_ld<V>(zw.r, e0 + r * st);
        } else {
#pragma unroll
            for (int r = 0; r < R0; ++r) v0[0][r] = buf_ld<V>(zw.r, (unsigned)zw.rel(np0 + r * nb0) * (unsigned)sizeof(V));
        }
        if constexpr (!EPI) {
            const __amdgpu_buffer_rsrc_t hr = buf_rsrc(H + sd.H_off, (unsigned)(M * sizeof(V)));
#pragma unroll
            for (int r = 0; r < R0; ++r)   // fused pass outputs j + r M/R0
                hreg[0][r] = buf_ld<V>(hr, (unsigned)(j + r * nb0) * (unsigned)sizeof(V));
        }
    }
    V* twL = L + k2_lds_data(g.k2_pts, SH);
    if constexpr (!NOPAD)
        for (int e = threadIdx.x; e < NTWF; e += K2_THREADS) twL[e] = twl[e];
    const auto twF = k2_tw_src<!NOPAD, V>(twL, twl);
    const auto twI = twF;   // palindrome: the reversed plan's table is the forward one
    constexpr int XZ = R0 == 16 ? 1 : 0;   // Ns = 1 outputs XOR-swizzled (see sh_store)
    shg_store<R0, false, NB0, SH, K2_THREADS, M, 1, XZ>(v0, rs, rows, StoreLds<V>{L}, tid);
    __syncthreads();
    K2_STAMP(1);
    shg_pass<R1, false, NB1, SH, K2_THREADS, M, NS1, CMP, XZ>(L, rs, rows, twF, StoreLds<V>{L});
    K2_STAMP(2);
    {
        V v[NB0][R0];
        shg_load<R0, false, NB0, SH, K2_THREADS, M, NS2, CMP>(L, rs, rows, twF + TW2, v, tid);
        RSP_WAR_SYNC();
        const __amdgpu_buffer_rsrc_t hr = buf_rsrc(H + sd.H_off, (unsigned)(M * sizeof(V)));
#pragma unroll
        for (int t = 0; t < NB0; ++t) {
            Dft<R0, false, V>::run(v[t]);
            if constexpr (EPI) {
                k2_apply_h<R0, nb0>(v[t], hr, j);   // fused pass outputs j + r M/R0
            } else {
#pragma unroll
                for (int r = 0; r < R0; ++r) v[t][r] = vmul(v[t][r], hreg[t][r]);
            }
        }
        shg_store<R0, true, NB0, SH, K2_THREADS, M, 1, XZ>(v, rs, rows, StoreLds<V>{L}, tid);
        __syncthreads();
    }
    K2_STAMP(3);
    shg_pass<R1, true, NB1, SH, K2_THREADS, M, NS1, CMP, XZ>(L, rs, rows, twI, StoreLds<V>{L});
    K2_STAMP(4);
    const int gend = min(sd.gb, g0 + sd.V);
    if constexpr (EPI) {
        shg_pass<R0, true, NB0, SH, K2_THREADS, M, NS2, CMP>(L, rs, rows, twI + TW2, StoreLds<V>{L});
        k2_epilogue<T, SH>(L, rs, rows, row0, rows_total, Lh1, g0, gend, rdm, mag, G, g.Gp);
    } else {
        static_assert(EPI || (rows == 1 && NS2 == nb0), "last pass: thread j's outputs are j + r NS2 of one row");
        V v[NB0][R0];
        shg_load<R0, true, NB0, SH, K2_THREADS, M, NS2, CMP>(L, rs, rows, twI + TW2, v, tid);
        if (rdm)
            shg_store<R0, true, NB0, SH, K2_THREADS, M, NS2>(
                v, rs, rows, StoreRowK<V, true, NS2, R0>(rdm, mag, G, g.Gp, row0, rows_total, Lh1, g0, gend), tid);
        else
            shg_store<R0, true, NB0, SH, K2_THREADS, M, NS2>(
                v, rs, rows, StoreRowK<V, false, NS2, R0>(rdm, mag, G, g.Gp, row0, rows_total, Lh1, g0, gend), tid);
    }
}

// k2_pc<T, WGS>: sized for WGS workgroups per CU.  WGS = 4 (a complex-double plan with a
// 2560-point block, Geometry::k2_pts = 2560: the row's 40 KB of LDS alone -- no pads, twiddles
// from L1/L2 (NOPAD) -- and 128 VGPRs per lane) runs the blocks with EPI (the filter spectrum loaded
// after the forward DFT, the kept gates stored by k2_epilogue): without them the last pass peaks
// at 188 VGPRs.  (Round 5's 3 per CU with pads and staged twiddles, 53.5 KB: 3 % slower.)
// WGS = 2 (4096-point workgroups, 76 KB of LDS) keeps H in registers from the start and stores
// the gates from the last pass, which measured faster at that occupancy (x2 at 2 per CU: 225 vs
// 248 us per 8 frames).
template <class T, int WGS>
__global__ __launch_bounds__(K2_THREADS, WGS) void k2_pc(Geometry g, DevConsts k, FramePtrs fp, int rows_total) {
    constexpr bool EPI = WGS >= 3;
    constexpr bool NOPAD = WGS == 4;
    typedef cx<T> V;
    V* L = reinterpret_cast<V*>(rsp_lds);   // overlap-save rows | narrow: staged rows + taps
    const int f = blockIdx.y;
    const int wg = k.k2order[blockIdx.x];   // the plan's dispatch order (job kinds interleaved)
    int ji = 0;
    while (ji + 1 < g.njobs && wg >= g.jobs[ji + 1].wg_begin) ++ji;
    const K2Job job = g.jobs[ji];
    const SegDesc& sd = g.segs[job.seg];
    const int rows = sd.rows_per_wg;
    const int row0 = (wg - job.wg_begin) * rows;
    const V* __restrict__ z = static_cast<const V*>(fp.z[f]);
    V* __restrict__ rdm = static_cast<V*>(fp.rdm[f]);
    T* __restrict__ mag = static_cast<T*>(fp.mag[f]);
    const int P = g.P, G = g.G;
    const int lo = sd.lo, hi = sd.hi, off = sd.off;
    const int tid = threadIdx.x;
    K2_STAMP(0);
    K2_TAG((unsigned long long)(sd.type * 16 + sd.logM));

    if (sd.type == 1 && sd.logM == 0) {   // mixed-radix block
        k2_fft_job_mix<T, 2560, 16, 10, EPI, NOPAD>(g, k, sd, job, z, rdm, mag, row0, rows_total, L);
    } else if (sd.type == 1) {
        if constexpr (WGS >= 3) {   // workgroups sized for the 2560-point block: 2048 points of 2^k rows
            static_assert(2048 <= 2560, "2^k rows in the 2560-point workgroup");
            switch (sd.logM) {
                case 6: k2_fft_job<T, 6, 2048, EPI, NOPAD>(g, k, sd, job, z, rdm, mag, row0, rows_total, L); break;
                case 7: k2_fft_job<T, 7, 2048, EPI, NOPAD>(g, k, sd, job, z, rdm, mag, row0, rows_total, L); break;
                case 8: k2_fft_job<T, 8, 2048, EPI, NOPAD>(g, k, sd, job, z, rdm, mag, row0, rows_total, L); break;
                case 9: k2_fft_job<T, 9, 2048, EPI, NOPAD>(g, k, sd, job, z, rdm, mag, row0, rows_total, L); break;
                case 10: k2_fft_job<T, 10, 2048, EPI, NOPAD>(g, k, sd, job, z, rdm, mag, row0, rows_total, L); break;
                default: k2_fft_job<T, 11, 2048, EPI, NOPAD>(g, k, sd, job, z, rdm, mag, row0, rows_total, L); break;
            }
        } else {
            switch (sd.logM) {
                case 6: k2_fft_job<T, 6, RSP_K2_POINTS, EPI, NOPAD>(g, k, sd, job, z, rdm, mag, row0, rows_total, L); break;
                case 7: k2_fft_job<T, 7, RSP_K2_POINTS, EPI, NOPAD>(g, k, sd, job, z, rdm, mag, row0, rows_total, L); break;
                case 8: k2_fft_job<T, 8, RSP_K2_POINTS, EPI, NOPAD>(g, k, sd, job, z, rdm, mag, row0, rows_total, L); break;
                case 9: k2_fft_job<T, 9, RSP_K2_POINTS, EPI, NOPAD>(g, k, sd, job, z, rdm, mag, row0, rows_total, L); break;
                case 10: k2_fft_job<T, 10, RSP_K2_POINTS, EPI, NOPAD>(g, k, sd, job, z, rdm, mag, row0, rows_total, L); break;
                case 11: k2_fft_job<T, 11, RSP_K2_POINTS, EPI, NOPAD>(g, k, sd, job, z, rdm, mag, row0, rows_total, L); break;
                default: k2_fft_job<T, 12, RSP_K2_POINTS, EPI, NOPAD>(g, k, sd, job, z, rdm, mag, row0, rows_total, L); break;
            }
        }
    } else {
        // direct FIR (narrow segment): filter() + circshift(-fir_delay) (fsf:111-112).  Each
        // staged row carries ntaps - 1 leading zeros (filter()'s zero state / samples before lo),
        // so the tap loop is branch-free.
        const int W = hi - lo + 1;
        const int PADL = sd.ntaps - 1, WP = W + PADL;
        const int nw = rows * WP;
        for (int e0 = 0; e0 < nw; e0 += 16 * K2_THREADS) {
            V val[16];
#pragma unroll
            for (int u = 0; u < 16; ++u) {
                const int e = e0 + tid + u * K2_THREADS;
                val[u] = V{};
                if (e < nw) {
                    const int rl = e / WP, i = e - rl * WP - PADL;
                    const int rho = row0 + rl;
                    if (rho < rows_total && i >= 0) {
                        const int b = rho / P, v = rho - b * P;
                        val[u] = z[zaddr(g, b, v, i + off)];
                    }
                }
            }
#pragma unroll
            for (int u = 0; u < 16; ++u) {
                const int e = e0 + tid + u * K2_THREADS;
                if (e < nw) L[e] = val[u];
            }
        }
        T* tp = reinterpret_cast<T*>(L + nw);   // taps: LDS broadcast reads
        const T* __restrict__ taps = static_cast<const T*>(k.taps);
        for (int e = tid; e < sd.ntaps; e += K2_THREADS) tp[e] = taps[sd.taps_off + e];
        __syncthreads();
        K2_STAMP(1);
        const int nout = sd.gb - sd.ga;
        // 4 consecutive gates per thread: the 4 outputs share a register window that slides one
        // sample per tap (1 LDS read + 4 FMAs per tap); a group whose circshift index wraps
        // mid-group takes the per-gate loop
        const int ngrp = (nout + 3) >> 2;
        for (int e = tid; e < rows * ngrp; e += K2_THREADS) {
            const int rl = e / ngrp, q0 = 4 * (e - rl * ngrp);
            const int rho = row0 + rl;
            if (rho >= rows_total) continue;
            const int gg0 = sd.ga + q0;
            int kk0 = (gg0 + sd.delay) % sd.Ls;
            if (kk0 < 0) kk0 += sd.Ls;
            const V* row = L + rl * WP + PADL - lo + sd.seg_lo;   // row[kk] = x(seg_lo + kk)
            if (q0 + 4 <= nout && kk0 + 3 < sd.Ls) {
                const V* xr = row + kk0;
                V w0 = xr[0], w1 = xr[1], w2 = xr[2], w3 = xr[3];
                T t = tp[0];
                V a0 = t * w0, a1 = t * w1, a2 = t * w2, a3 = t * w3;
#pragma unroll 4
                for (int j = 1; j < sd.ntaps; ++j) {
                    w3 = w2; w2 = w1; w1 = w0;
                    w0 = xr[-j];
                    t = tp[j];
                    a0 += t * w0; a1 += t * w1; a2 += t * w2; a3 += t * w3;
                }
                if (rdm) {
                    V* ro = rdm + (size_t)rho * G + gg0;
                    ro[0] = a0; ro[1] = a1; ro[2] = a2; ro[3] = a3;
                }
                T* mo = mag + (size_t)rho * g.Gp + gg0;
                mo[0] = cmag(a0); mo[1] = cmag(a1); mo[2] = cmag(a2); mo[3] = cmag(a3);
            } else {
                for (int q = 0; q < 4 && q0 + q < nout; ++q) {
                    const int gg = gg0 + q;
                    int kk = (gg + sd.delay) % sd.Ls;
                    if (kk < 0) kk += sd.Ls;
                    const V* xr = row + kk;
                    V acc = V{};
                    for (int j = 0; j < sd.ntaps; ++j) acc += tp[j] * xr[-j];
                    if (rdm) rdm[(size_t)rho * G + gg] = acc;
                    mag[(size_t)rho * g.Gp + gg] = cmag(acc);
                }
            }
        }
    }
    K2_STAMP(5);
}

// ======================================================================================
// K3: GOCA-CFAR on adjacent-beam sums + compaction + S9 estimation
// ======================================================================================
// Peak of MATLAB interp1(...,'spline') (not-a-knot) sampled at step 1/interp over n
// equally spaced points (fsf:257-260, 272-275); returns the first-argmax abscissa.
template <int INTERP>
__device__ __forceinline__ double spline_peak(const double* y, int n) {
    // Piecewise-cubic coefficients per unit interval, then Horner at q / INTERP; the sample
    // grid and the first-argmax rule are the reference's (interp1 on cells(1):1/INTERP:cells(end)).
    constexpr double dx = 1.0 / INTERP;   // 1/8, 1/4: exact
    double c0[4], c1[4], c2[4], c3[4];   // value on [i, i+1]: ((c3 t + c2) t + c1) t + c0
    if (n == 5) {   // not-a-knot second derivatives, unit spacing (closed form of the 5x5 system)
        double Mv[5];
        Mv[1] = y[0] - 2.0 * y[1] + y[2];
        Mv[3] = y[2] - 2.0 * y[3] + y[4];
        Mv[2] = (6.0 * (y[1] - 2.0 * y[2] + y[3]) - Mv[1] - Mv[3]) * 0.25;
        Mv[0] = 2.0 * Mv[1] - Mv[2];
        Mv[4] = 2.0 * Mv[3] - Mv[2];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            c0[i] = y[i];
            c1[i] = (y[i + 1] - y[i]) - (2.0 * Mv[i] + Mv[i + 1]) * (1.0 / 6.0);
            c2[i] = 0.5 * Mv[i];
            c3[i] = (Mv[i + 1] - Mv[i]) * (1.0 / 6.0);
        }
    } else {          // n == 4: the single cubic through 4 points; n == 3: the parabola
        const double d1 = y[1] - y[0], d2_ = y[2] - 2.0 * y[1] + y[0];
        const double d3 = (n == 4) ? y[3] - 3.0 * y[2] + 3.0 * y[1] - y[0] : 0.0;
        // Newton form about x = 0 expanded at each integer knot i
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const double x = i;
            c0[i] = y[0] + x * d1 + x * (x - 1.0) * 0.5 * d2_ + x * (x - 1.0) * (x - 2.0) * (1.0 / 6.0) * d3;
            c1[i] = d1 + (2.0 * x - 1.0) * 0.5 * d2_ + (3.0 * x * x - 6.0 * x + 2.0) * (1.0 / 6.0) * d3;
            c2[i] = 0.5 * d2_ + (3.0 * x - 3.0) * (1.0 / 6.0) * d3;
            c3[i] = (1.0 / 6.0) * d3;
        }
    }
    // samples q = 0 .. (n-1) INTERP in order (first argmax wins); sample q lies on interval
    // min(q / INTERP, n - 2) like ppval -- every array index is a compile-time constant
    double best = -INFINITY, bx = 0.0;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        if (i < n - 1) {
#pragma unroll
            for (int t = 0; t < INTERP; ++t) {
                const double tt = t * dx;
                const double val = ((c3[i] * tt + c2[i]) * tt + c1[i]) * tt + c0[i];
                if (val > best) {
                    best = val;
                    bx = (i * INTERP + t) * dx;
                }
            }
        }
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {   // the last sample: end of the last interval
        if (i == n - 2) {
            const double val = ((c3[i] + c2[i]) + c1[i]) + c0[i];
            if (val > best) bx = (n - 1);
        }
    }
    return bx;
}

// The axes, angles and K-LUT S9 reads (DevConsts fields), by value so that the out-of-line
// spill path below takes them in registers.
struct S9Consts {
    const double *range_axis, *velocity_axis, *beam_angles, *klut;
    double deltaR, deltaV;
};

// S9 of one detection from the workgroup's S tile (fsf:237-290).
// sval(v, r) = S at Doppler row v, range cell r (the tile, or the maps when the tile lacks it).
// RA / RB (RSP_PLAN_MONOPULSE_COMPLEX, else null): the complex RD map rows of beams pair, pair + 1.
template <class T, class SF>
__device__ __forceinline__ void s9_estimate(const S9Consts& k, SF sval, int P, int G, int Gp, int v, int r, int pair,
                                            const T* __restrict__ MA, const T* __restrict__ MB,
                                            const cx<T>* __restrict__ RA, const cx<T>* __restrict__ RB, DevDet* out) {
    // the 5-cell windows clipped to the map (fsf:241-250): cells first .. first + n - 1
    const int rfirst = max(r - 2, 0), nrc = min(r + 2, G - 1) - rfirst + 1;
    const int vfirst = max(v - 2, 0), nvc = min(v + 2, P - 1) - vfirst + 1;
    double yr[5], yv[5];
#pragma unroll
    for (int j = 0; j < 5; ++j) {
        yr[j] = j < nrc ? (double)sval(v, rfirst + j) : 0.0;
        yv[j] = j < nvc ? (double)sval(vfirst + j, r) : 0.0;
    }
    const double rmax = (nrc < 3) ? (double)r : rfirst + spline_peak<8>(yr, nrc);
    const double vmax = (nvc < 3) ? (double)v : vfirst + spline_peak<4>(yv, nvc);
    double ratio;
    if (RA) {   // complex ratio real((S_A - S_B) / (S_A + S_B + eps)) (main_plot_snr_vs_angle_error.m:455-462)
        const cx<T> a = RA[(size_t)v * G + r], b = RB[(size_t)v * G + r];
        const double nx = (double)a.x - (double)b.x, ny = (double)a.y - (double)b.y;
        const double dx = (double)a.x + (double)b.x + 2.220446049250313e-16, dy = (double)a.y + (double)b.y;
        ratio = (nx * dx + ny * dy) / (dx * dx + dy * dy);
    } else {    // amplitude monopulse on the integer cell (fsf:282-290)
        const double SA = (double)MA[(size_t)v * Gp + r];
        const double SB = (double)MB[(size_t)v * Gp + r];
        ratio = (SA - SB) / (SA + SB + 2.220446049250313e-16);
    }
    DevDet d;
    d.v_idx = v + 1;
    d.r_idx = r + 1;
    d.pair_idx = pair + 1;
    d.reserved = 0;
    d.amp = (double)sval(v, r);
    d.range = k.range_axis[r] + (rmax - r) * k.deltaR;
    d.velocity = k.velocity_axis[v] + (vmax - v) * k.deltaV;
    d.angle = 0.5 * (k.beam_angles[pair] + k.beam_angles[pair + 1]) + k.klut[pair] * ratio;
    *out = d;
}

#define K3_QCAP 1024

#define K3_VEC 8       // 16-B loads per beam per thread in flight (halo-less 98-row tiles: 8 -> 120 rows per sweep)
#define RSP_K3_WGS 3   // k3_cfar workgroups per CU the register budget is sized for

constexpr int floor4(int x) { return x >= 0 ? (x & ~3) : -((-x + 3) & ~3); }

// 4 consecutive cells of an S row from LDS (16-B aligned): one ds_read_b128 (float) or two
// (double)
__device__ __forceinline__ void ld4(const float* p, float (&o)[4]) {
    const f32x4 t = *reinterpret_cast<const f32x4*>(p);
    o[0] = t.x; o[1] = t.y; o[2] = t.z; o[3] = t.w;
}
__device__ __forceinline__ void ld4(const double* p, double (&o)[4]) {
    const d2 a = *reinterpret_cast<const d2*>(p), b = *reinterpret_cast<const d2*>(p + 2);
    o[0] = a.x; o[1] = a.y; o[2] = b.x; o[3] = b.y;
}
template <class T> struct U16;   // one 16-B unit of a map row
template <> struct U16<float> { typedef f32x4 U; static constexpr int E = 4; };
template <> struct U16<double> { typedef d2 U; static constexpr int E = 2; };

// RR/RV/GR/GV = reference/guard cell counts when known at compile time (the reference's
// 5/5/10/10, v8:45-46), 0 = runtime; RTC = the tile width g.cfar_RT when they are (32 or 64),
// so that the LDS row stride and every window offset are compile-time constants.  Tiles: RT
// range cells x all P Doppler cells of one beam pair, tile starts aligned to 4 cells so that
// the magnitude rows load as 16-B units.
template <class T, int RR, int RV, int GR, int GV, int RTC>
__global__ __launch_bounds__(RSP_THREADS, RSP_K3_WGS) void k3_cfar(Geometry g, DevConsts k, FramePtrs fp) {
    T* S = reinterpret_cast<T*>(rsp_lds);   // [P][W] | queue[K3_QCAP] | qn, base
    typedef typename U16<T>::U U;
    constexpr int EPU = U16<T>::E;
    constexpr bool FAST = RR > 0 && RV > 0 && GR > 0 && GV > 0 && (RTC == 32 || RTC == 64);
    constexpr int HRC = ((RR + GR > 2 ? RR + GR : 2) + 3) & ~3;   // = g.cfar_hR (rsp_plan.cpp)
    // = g.cfar_W; complex double rows get 2 extra cells (stride 132 dwords = 4 mod 64 banks), see
    // the row-group order of the CFAR loop
    // NOH (the fast path): the tile holds the band's own cells only, no halo; the
    // prefilter takes whichever range slice lies inside the tile, survivors and S9 read the rest
    // from the maps
    constexpr bool NOH = FAST;
    constexpr int WC = ((RTC + (NOH ? 0 : 2) * HRC + 3) & ~3) + (sizeof(T) == 8 ? 2 : 0);
    // XCD-aware order (bijective swizzle, cdna_hip_programming.md T1): the workgroups that
    // share an XCD take consecutive (tile, pair) ids with pairs fastest, so beam b's tile --
    // read by pairs b-1 and b -- and the range halos of neighbouring tiles are L2 hits
    const int npair = g.B - 1, ntile = k3_ntiles(g);
    int wg = blockIdx.x;
    {
        const int nwg = gridDim.x, xcd = wg & 7, q = nwg >> 3, rm = nwg & 7;
        wg = (xcd < rm ? xcd * (q + 1) : rm * (q + 1) + (xcd - rm) * q) + (wg >> 3);
    }
    const int pair = wg % npair, col = wg / npair;
    const int tile = col % ntile, col2 = col / ntile;
    const int band = col2 % g.cfar_nband, f = col2 / g.cfar_nband;
    const int P = g.P, G = g.G, W = FAST ? WC : g.cfar_W, hR = FAST ? HRC : g.cfar_hR, RT = FAST ? RTC : g.cfar_RT;
    const int rR = RR ? RR : g.refR, gR = GR ? GR : g.guardR, rV = RV ? RV : g.refV, gV = GV ? GV : g.guardV;
    const int rc0 = rR + gR;                           // first cell under test (0-based)
    const int tstart = (rc0 & ~3) + tile * RT;         // multiple of 4
    const int c0 = tstart - (NOH ? 0 : hR);            // tile column 0 (multiple of 4; may be < 0)
    const int cut_lo = max(tstart, rc0), cut_hi = min(tstart + RT, G - rc0);
    // Doppler band: cells under test in rows [v0, v1), the tile holds rows [vt0, vt1) (the
    // band plus the rV + gV window rows on each side; bands of one tile column tile the map)
    const int hV = rV + gV;
    const int v0 = hV + band * g.cfar_VB, v1 = min(hV + (band + 1) * g.cfar_VB, P - hV);
    const int vt0 = NOH ? v0 : max(v0 - hV, 0), vt1 = NOH ? max(v1, v0) : min(v1 + hV, P), nv = vt1 - vt0;
    int* queue = reinterpret_cast<int*>(S + g.cfar_rows * W);
    int* qn = queue + K3_QCAP;
    const T* Sv = S - vt0 * W;                         // row v of the map at Sv + v W
    const int Gp = g.Gp;
    const T* __restrict__ MA = static_cast<const T*>(fp.mag[f]) + (size_t)pair * P * Gp;   // |RDM| of beams pair, pair+1
    const T* __restrict__ MB = MA + (size_t)P * Gp;
    const cx<T>* __restrict__ RA = g.mono_c ? static_cast<const cx<T>*>(fp.rdm[f]) + (size_t)pair * P * G : nullptr;
    const cx<T>* __restrict__ RB = RA ? RA + (size_t)P * G : nullptr;
    // S(v, r) from the maps: the same two values and the same add as the tile load below
    auto sg = [&](int vv, int rr) -> T {
        const size_t o = (size_t)vv * Gp + rr;
        return MA[o] + MB[o];
    };
    if (threadIdx.x == 0) qn[0] = 0;
    // ---- load S = |A| + |B| (fsf:184-187) from the magnitude maps: 16 B per lane,
    //      K3_VEC units of each beam in flight per thread
    if constexpr (FAST) {
        // a thread keeps one 16-B column unit and walks the rows: one address add per load
        constexpr int WU = WC / EPU, NTR = RSP_THREADS / WU;
        const int u = threadIdx.x % WU, rr = threadIdx.x / WU;
        const int r = c0 + EPU * u;
        const bool colok = rr < NTR && r >= 0 && r < G;   // rows are padded to Gp: r + EPU - 1 < Gp
        const T* pa = MA + (size_t)(vt0 + rr) * Gp + r;
        const T* pb = MB + (size_t)(vt0 + rr) * Gp + r;
        U* sd = reinterpret_cast<U*>(S + rr * WC) + u;
        // complex single: the two maps as buffer resources, a unit outside the tile gets an
        // out-of-range offset (bit 31) and reads 0 -- no branch around a load, so the 2 K3_VEC
        // loads of a sweep are in flight together
        const unsigned mbytes = (unsigned)((size_t)P * Gp * sizeof(T));
        const __amdgpu_buffer_rsrc_t ra = buf_rsrc(MA, mbytes), rbm = buf_rsrc(MB, mbytes);
        const unsigned base = colok ? (unsigned)(((size_t)(vt0 + rr) * Gp + r) * sizeof(T)) : RSP_OOB;
        const unsigned rowb = (unsigned)Gp * (unsigned)sizeof(T);
        for (int vb = 0; vb < nv; vb += K3_VEC * NTR) {
            U xa[K3_VEC], xb[K3_VEC];
#pragma unroll
            for (int q = 0; q < K3_VEC; ++q) {
                if constexpr (sizeof(T) == 4) {   // complex double: plain loads (35.0 vs 36.0 us)
                    const unsigned bad = (unsigned)(nv - 1 - (vb + rr + q * NTR)) & 0x80000000u;
                    const unsigned off = (base + (unsigned)(vb + q * NTR) * rowb) | bad;
                    xa[q] = __builtin_bit_cast(U, __builtin_amdgcn_raw_buffer_load_b128(ra, (int)off, 0, 0));
                    xb[q] = __builtin_bit_cast(U, __builtin_amdgcn_raw_buffer_load_b128(rbm, (int)off, 0, 0));
#pragma unroll
                    for (int e = 1; e < EPU; ++e)   // the row pad past G (Gp > G) is not written by K2
                        if (r + e >= G) { xa[q][e] = 0; xb[q][e] = 0; }
                    continue;
                }
                xa[q] = U{};
                xb[q] = xa[q];
                if (colok && vb + rr + q * NTR < nv) {
                    xa[q] = *reinterpret_cast<const U*>(pa + (size_t)(vb + q * NTR) * Gp);
                    xb[q] = *reinterpret_cast<const U*>(pb + (size_t)(vb + q * NTR) * Gp);
#pragma unroll
                    for (int e = 1; e < EPU; ++e)
                        if (r + e >= G) { xa[q][e] = 0; xb[q][e] = 0; }
                }
            }
#pragma unroll
            for (int q = 0; q < K3_VEC; ++q)
                if (rr < NTR && vb + rr + q * NTR < nv) sd[(vb + q * NTR) * WU] = xa[q] + xb[q];
        }
    } else {
        const int WU = W / EPU, nu = nv * WU;
        for (int e0 = 0; e0 < nu; e0 += K3_VEC * RSP_THREADS) {
            U xa[K3_VEC], xb[K3_VEC];
#pragma unroll
            for (int u = 0; u < K3_VEC; ++u) {
                const int e = e0 + threadIdx.x + u * RSP_THREADS;
                xa[u] = U{};
                xb[u] = xa[u];
                if (e < nu) {
                    const int vl = e / WU, r = c0 + EPU * (e - vl * WU), v = vt0 + vl;
                    if (r >= 0 && r < G) {   // rows are padded to Gp (multiple of 4): r + EPU - 1 < Gp
                        xa[u] = *reinterpret_cast<const U*>(MA + (size_t)v * Gp + r);
                        xb[u] = *reinterpret_cast<const U*>(MB + (size_t)v * Gp + r);
#pragma unroll
                        for (int q = 1; q < EPU; ++q)
                            if (r + q >= G) { xa[u][q] = 0; xb[u][q] = 0; }
                    }
                }
            }
#pragma unroll
            for (int u = 0; u < K3_VEC; ++u) {
                const int e = e0 + threadIdx.x + u * RSP_THREADS;
                if (e < nu) reinterpret_cast<U*>(S)[e] = xa[u] + xb[u];
            }
        }
    }
    __syncthreads();
    if (fp.smap[f]) {   // on request: rdm_for_cfar_all as thresholded here, [pair][v][r]
        T* sm = static_cast<T*>(fp.smap[f]) + (size_t)pair * P * G;
        const int wlo = tile == 0 ? 0 : tstart, whi = tile == ntile - 1 ? G : min(tstart + RT, G);
        const int vlo = band == 0 ? 0 : v0, vhi = band == g.cfar_nband - 1 ? P : v1;   // inside [vt0, vt1)
        const int nwc = whi - wlo;
        for (int e = threadIdx.x; e < (vhi - vlo) * nwc; e += RSP_THREADS) {
            const int v = vlo + e / nwc, r = wlo + (e - (v - vlo) * nwc);
            sm[(size_t)v * G + r] = NOH ? sg(v, r) : Sv[v * W + (r - c0)];
        }
    }
    if (v1 <= v0 || cut_hi <= cut_lo) return;
    const double Tc = g.T;
    // mean() = sum / n over the slices of fsf:197-203 (max(a/n, b/n) = max(a, b)/n).  double: the
    // correctly rounded quotient, as MATLAB, without a division: q0 = x * RN(1/n), r = x - q0 n
    // (exact, one FMA), q = RN(q0 + r RN(1/n)) is RN(x/n) (Markstein's theorem: RN(1/n) within half
    // an ulp, q0 within one ulp of x/n; no underflow for these sums).  float: a multiply by 1/n
    // (<= 1 ulp from the quotient).  With n_R = n_V (the reference's 5/5) max(nR, nV) is one
    // quotient of the largest slice sum.
    const T fR = (T)rR, fV = (T)rV;
    const T iR = (T)1 / fR, iV = (T)1 / fV;
    auto quot = [&](T x, T fn, T in) -> T {
        if constexpr (sizeof(T) == 8) {
            const T q0 = x * in;
            return __builtin_fma(__builtin_fma(-q0, fn, x), in, q0);
        } else {
            return x * in;
        }
    };
    auto noise2 = [&](T lr, T tr, T lv, T tv) -> T {
        if (FAST && RR == RV) return quot(fmax(fmax(lr, tr), fmax(lv, tv)), fR, iR);
        const T nR = quot(fmax(lr, tr), fR, iR), nV = quot(fmax(lv, tv), fV, iV);
        return nR > nV ? nR : nV;
    };
    const S9Consts s9c{k.range_axis, k.velocity_axis, k.beam_angles, k.klut, k.deltaR, k.deltaV};
    // hits past the LDS queue are only counted here (qn keeps counting); the overflow pass below
    // finds them again
#define K3_HIT(V, C, CUT, LR, TR, LV, TV)                                                               \
    do {                                                                                                \
        if ((CUT) > (T)Tc * noise2(LR, TR, LV, TV)) {                                                   \
            const int qi = atomicAdd(qn, 1);                                                            \
            if (qi < K3_QCAP) queue[qi] = ((V) << 16) | (C);                                            \
        }                                                                                               \
    } while (0)
    // ---- cross GOCA-CFAR (fsf:192-213); hits go to an LDS queue so that the S9 work is
    //      spread over the whole workgroup instead of serialising in the lane that owns a range cell
    if constexpr (FAST) {   // RT = 32: long-P / double tiles (LDS cap in the plan)
        // a thread takes 4 adjacent range cells of one Doppler row: every window value comes
        // from 16-B LDS reads; sums run left to right over each slice like mean()
        constexpr int DL = -(GR + RR), DR = GR + 1;              // window starts rel. to the cell
        constexpr int BL = floor4(DL), BR = floor4(DR);
        constexpr int NL = (DL + 3 + RR - BL + 3) / 4, NR = (DR + 3 + RR - BR + 3) / 4;
        constexpr int lgT = RTC == 64 ? 4 : 3;                    // log2 threads per row (RT / 4)
        // 16-lane row groups of a wave take rows {0, 2, 1, 3} + 4w: the ds_read_b128 lane groups
        // ({0-3,12-15,20-27}, ... MI355X_MICROARCH.md §LDS) then pair rows 2 apart, 2W = 192
        // floats = 0 mod 64 banks, conflict-free (adjacent rows, W = 96 = 32 mod 64, were 2-way)
        const int rg = threadIdx.x >> lgT;
        // complex double (8 threads per row, 32 B per thread, two ds_read_b128 of 16 lanes from 4
        // row groups; row stride 34 doubles, so a 16-B slot's bank is (row + 2 q + base / 2) mod
        // 16 slots): row groups 4a + {0, 1, 2, 3} take rows {0, 1, 8, 9} + 2 (a mod 4) + 16 (a / 4),
        // and their column groups q are rotated by {0, 4, 4, 0}, so that each ds_read_b128 lane
        // group holds four rows {0, 1, 8, 9} (+ x) of ONE half of the columns (q < 4 or q >= 4).
        // Every lane of a group then reads at the same offset (the halo-less prefilter's right
        // slice is read by q < 4 only, the left one by q >= 4), and rows + 2 q cover the 16 slots
        // once.  (Rows 2a + {0, 16, 1, 17} with unrotated columns put the two slices in one lane
        // group: 2-way on a quarter of the slots, 30 % of K3's LDS cycles.)
        const int q = lgT == 3 ? ((threadIdx.x & 7) ^ (((rg ^ (rg >> 1)) & 1) << 2)) : threadIdx.x & ((1 << lgT) - 1);
        const int c = (NOH ? 0 : hR) + 4 * q;                     // first tile column of the group
        const int r = c0 + c;
        const int rgp = lgT == 4 ? (rg & ~3) | ((rg & 1) << 1) | ((rg >> 1) & 1)
                                 : (rg & 1) + ((rg & 2) << 2) + 2 * ((rg >> 2) & 3) + 16 * (rg >> 4);
        // Exact prefilter.  A hit needs CUT > T mean(max of the four slices) >= T mean(left range
        // slice): quot() is the correctly rounded (double) or a monotone (float) quotient and the
        // product with T > 0 rounds monotonically, so a cell with CUT <= T quot(lr) cannot be a
        // hit.  That test needs the left range slice alone (4 of the 27 ld4 per 4 cells: the CFAR
        // phase was bound by LDS bandwidth); the rare survivors (T = 8 on amplitude sums: cells
        // near targets) run the full test below with the same sums in the same order, so the
        // detection list is the one the full test gives.  A NaN sum never rejects (the
        // comparison is false).
        if (NOH || Tc > 0.0) {
            const T Tt = (T)Tc;
            const bool pf = Tc > 0.0;   // the bound needs T > 0; otherwise every cell takes the full test
            // NOH: lanes whose 4 cells start in the first 16 tile columns test the right range
            // slice (cells c + 11 .. c + 15 + 3 <= 30 < RT), the others the left one (c - 15 >= 1):
            // either is a lower bound of the max.  The right slice's loads start at c + OR so
            // that both slices sit at the same register offsets when the alignment allows (ld4 of
            // double: 2 cells; of float: 4 cells, so float selects between offsets 1 and 3)
            static_assert(!NOH || (RR == 5 && GR == 10 && NL == 3 && BL == -16), "NOH constants for the 5/10 window");
            constexpr int OR = sizeof(T) == 8 ? 10 : 8, XR = DR - OR;   // XR: register offset of the right slice
            const bool useR = NOH && q < 4;
            const int base = useR ? OR : BL;
#pragma unroll 1
            for (int v = v0 + rgp; v < v1; v += RSP_THREADS >> lgT) {
                const T* row = Sv + v * WC + c;
                T xl[4 * NL], cv[4];
#pragma unroll
                for (int j = 0; j < NL; ++j) {
                    T t[4];
                    ld4(row + base + 4 * j, t);
#pragma unroll
                    for (int i = 0; i < 4; ++i) xl[4 * j + i] = t[i];
                }
                ld4(row, cv);
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    T lr = 0;   // NOH: the left or the right slice sum (a lower bound either way)
#pragma unroll
                    for (int qq = 0; qq < RR; ++qq) {
                        const T xa = xl[i + DL - BL + qq];
                        if constexpr (NOH && XR != DL - BL) lr += useR ? xl[i + XR + qq] : xa;
                        else lr += xa;
                    }
                    const int ri = r + i;
                    if (ri >= cut_lo && ri < cut_hi && (!pf || !(cv[i] <= Tt * quot(lr, fR, iR)))) {
                        T tr = 0, lv = 0, tv = 0;
                        if constexpr (NOH) {   // every slice from the maps, in sum() order
                            lr = 0;
                            for (int qq = 0; qq < RR; ++qq) lr += sg(v, ri + DL + qq);
                            for (int qq = 0; qq < RR; ++qq) tr += sg(v, ri + DR + qq);
                            for (int qq = 0; qq < RV; ++qq) {
                                lv += sg(v + qq - GV - RV, ri);
                                tv += sg(v + qq + GV + 1, ri);
                            }
                        } else {
                            const T* cp = row + i;
#pragma unroll
                            for (int qq = 0; qq < RR; ++qq) tr += cp[DR + qq];
#pragma unroll
                            for (int qq = 0; qq < RV; ++qq) {
                                lv += cp[(qq - GV - RV) * WC];
                                tv += cp[(qq + GV + 1) * WC];
                            }
                        }
                        K3_HIT(v, c + i, cv[i], lr, tr, lv, tv);
                    }
                }
            }
        } else
#pragma unroll 1
        for (int v = v0 + rgp; v < v1; v += RSP_THREADS >> lgT) {
            const T* row = Sv + v * WC + c;
            T xl[4 * NL], xr[4 * NR], cv[4];
            T lv[4] = {0, 0, 0, 0}, tv[4] = {0, 0, 0, 0};
#pragma unroll
            for (int j = 0; j < NL; ++j) {
                T t[4];
                ld4(row + BL + 4 * j, t);
#pragma unroll
                for (int i = 0; i < 4; ++i) xl[4 * j + i] = t[i];
            }
#pragma unroll
            for (int j = 0; j < NR; ++j) {
                T t[4];
                ld4(row + BR + 4 * j, t);
#pragma unroll
                for (int i = 0; i < 4; ++i) xr[4 * j + i] = t[i];
            }
            ld4(row, cv);
#pragma unroll
            for (int qq = 0; qq < RV; ++qq) {
                T a[4], b[4];
                ld4(row + (qq - GV - RV) * WC, a);
                ld4(row + (qq + GV + 1) * WC, b);
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    lv[i] += a[i];
                    tv[i] += b[i];
                }
            }
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                T lr = 0, tr = 0;
#pragma unroll
                for (int qq = 0; qq < RR; ++qq) {
                    lr += xl[i + DL - BL + qq];
                    tr += xr[i + DR - BR + qq];
                }
                const int ri = r + i;
                if (ri >= cut_lo && ri < cut_hi) K3_HIT(v, c + i, cv[i], lr, tr, lv[i], tv[i]);
            }
        }
    } else {
        const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;   // 4 waves
        for (int rb = cut_lo; rb < cut_hi; rb += 64) {
            const int r = rb + lane;
            if (r >= cut_hi) continue;
            const int c = r - c0;
            for (int v = v0 + wv; v < v1; v += 4) {
                const T* rowp = Sv + v * W;
                T lr = 0, tr = 0, lv = 0, tv = 0;
                const T* lrp = rowp + c - gR - rR;
                const T* trp = rowp + c + gR + 1;
                const T* lvp = Sv + (v - gV - rV) * W + c;
                const T* tvp = Sv + (v + gV + 1) * W + c;
                for (int qq = 0; qq < rR; ++qq) {
                    lr += lrp[qq];
                    tr += trp[qq];
                }
                for (int qq = 0; qq < rV; ++qq) {
                    lv += lvp[qq * W];
                    tv += tvp[qq * W];
                }
                K3_HIT(v, c, rowp[c], lr, tr, lv, tv);
            }
        }
    }
#undef K3_HIT
    __syncthreads();
    const int nhit = qn[0], n = min(nhit, K3_QCAP);
    if (n == 0) return;
    if (threadIdx.x == 0) qn[1] = atomicAdd(fp.count[f], n);   // one global reservation per workgroup
    __syncthreads();
    const int base = qn[1];
    // S(v, r) as the CFAR test read it: the tile, or the maps where a halo-less tile lacks it
    auto st = [&](int vv, int rr) -> T {
        if constexpr (NOH) return sg(vv, rr);
        else return Sv[vv * W + (rr - c0)];
    };
    for (int i = threadIdx.x; i < n; i += RSP_THREADS) {
        const int idx = base + i;
        if (idx >= g.max_dets) break;   // counted; the host grows the list and runs K3 again
        const int e = queue[i];
        const int v = e >> 16, c = e & 0xFFFF;
        s9_estimate<T>(s9c, st, P, G, Gp, v, c0 + c, pair, MA, MB, RA, RB, &fp.dets[f][idx]);
    }
    if (nhit <= K3_QCAP) return;   // uniform
    // Overflow pass (more than K3_QCAP hits in this tile: a cluttered frame or a low T_CFAR).  The
    // list holds every hit, like all_raw_detections(end+1, :) (fsf:215-221): the queued cells are
    // marked in a bitmap over the tile's cells under test (in the queue's LDS), and every other
    // cell is tested again, with the same sums in the same order as above, so the same cells hit;
    // each unmarked hit reserves its slot and runs S9.  Outside the CFAR loop, so the common path
    // keeps its registers and schedule (an in-loop spill call cost K3 25 %).
    constexpr int HELD = K3_QCAP / RSP_THREADS;
    int held[HELD];
#pragma unroll
    for (int u = 0; u < HELD; ++u) held[u] = queue[threadIdx.x + u * RSP_THREADS];
    __syncthreads();
    unsigned* bm = reinterpret_cast<unsigned*>(queue);   // ncr x (v1 - v0) bits <= K3_QCAP x 32
    const int ncr = cut_hi - cut_lo, ncell = (v1 - v0) * ncr;
#pragma unroll
    for (int u = 0; u < HELD; ++u) bm[threadIdx.x + u * RSP_THREADS] = 0u;
    __syncthreads();
#pragma unroll
    for (int u = 0; u < HELD; ++u) {
        const int v = held[u] >> 16, r = c0 + (held[u] & 0xFFFF);
        const int bit = (v - v0) * ncr + (r - cut_lo);
        atomicOr(&bm[bit >> 5], 1u << (bit & 31));
    }
    __syncthreads();
    for (int e = threadIdx.x; e < ncell; e += RSP_THREADS) {
        if (bm[e >> 5] >> (e & 31) & 1u) continue;
        const int v = v0 + e / ncr, r = cut_lo + (e - (e / ncr) * ncr);
        T lr = 0, tr = 0, lv = 0, tv = 0;
        for (int qq = 0; qq < rR; ++qq) {
            lr += st(v, r - gR - rR + qq);
            tr += st(v, r + gR + 1 + qq);
        }
        for (int qq = 0; qq < rV; ++qq) {
            lv += st(v + qq - gV - rV, r);
            tv += st(v + qq + gV + 1, r);
        }
        if (st(v, r) > (T)Tc * noise2(lr, tr, lv, tv)) {
            const int idx = atomicAdd(fp.count[f], 1);
            if (idx < g.max_dets) s9_estimate<T>(s9c, st, P, G, Gp, v, r, pair, MA, MB, RA, RB, &fp.dets[f][idx]);
        }
    }
}

// ======================================================================================
// MTD over pulses of a pulse-compressed cube pc[B][P][G] -> rdm[B][P][G] (fsf:131-136)
// ======================================================================================
template <class T, int LGP>
__global__ __launch_bounds__(RSP_THREADS, 2) void k_mtd_cols(Geometry g, DevConsts k, const cx<T>* __restrict__ pc,
                                                        cx<T>* __restrict__ rdm) {
    typedef cx<T> V;
    V* Y = reinterpret_cast<V*>(rsp_lds);   // [GT][Ppad] + W_P table
    constexpr int GT = 16;
    V* twl = Y + GT * g.Ppad;
    const T* __restrict__ win = static_cast<const T*>(k.win);
    if constexpr (LGP > 0)
        for (int i = threadIdx.x; i < tw_total(LGP); i += RSP_THREADS) twl[i] = static_cast<const V*>(k.twPp)[i];
    const int b = blockIdx.y, gt0 = blockIdx.x * GT;
    const int P = g.P, G = g.G, Ppad = g.Ppad;
    for (int e = threadIdx.x; e < P * GT; e += RSP_THREADS) {
        const int m = e / GT, gl = e - m * GT;
        const int gg = gt0 + gl;
        V val = V{};
        if (gg < G) val = pc[((size_t)b * P + m) * G + gg] * win[m];
        Y[gl * Ppad + m] = val;
    }
    __syncthreads();
    const int half = P >> 1;
    if constexpr (LGP > 0) {
        StoreLds<V> st{Y};
        fft_passes<LGP, (16 << LGP) / RSP_THREADS, 0, RSP_THREADS>(Y, Ppad, GT, twl, st, st);
        for (int e = threadIdx.x; e < P * GT; e += RSP_THREADS) {
            const int v = e / GT, gl = e - v * GT;
            const int gg = gt0 + gl;
            int src = v - half;
            if (src < 0) src += P;
            if (gg < G) rdm[((size_t)b * P + v) * G + gg] = Y[gl * Ppad + src];
        }
    } else {
        const V* __restrict__ twP = static_cast<const V*>(k.twP);
        for (int e = threadIdx.x; e < P * GT; e += RSP_THREADS) {
            const int v = e / GT, gl = e - v * GT;
            const int gg = gt0 + gl;
            int kk = v - half;
            if (kk < 0) kk += P;
            V acc = V{};
            int idx = 0;
            for (int p = 0; p < P; ++p) {
                acc += vmul(Y[gl * Ppad + p], twP[idx]);
                idx += kk;
                if (idx >= P) idx -= P;
            }
            if (gg < G) rdm[((size_t)b * P + v) * G + gg] = acc;
        }
    }
}

// ======================================================================================
// S4 + S4.1 on the device: echo synthesis + Philox noise (fsf:45-88)
// ======================================================================================
// The per-target phasors of S4, once per (target, pulse) and (target, channel) instead of once per
// sample: tab[t][j] = e^{i 2 pi fd_prt j} for j < P (doppler_phase_shift, fsf:58), then
// e^{i c dphi} for c < C (the channel phasor, fsf:71-72) -- the same sincos arguments, so the
// cube is what the per-sample evaluation gave.
__global__ __launch_bounds__(RSP_THREADS) void k_synth_tab(Geometry g, SynthTargets tg, int nt, d2* __restrict__ tab) {
    const int per = g.P + g.C;
    const int i = blockIdx.x * RSP_THREADS + threadIdx.x;
    if (i >= nt * per) return;
    const int t = i / per, j = i - t * per;
    double s, c;
    if (j < g.P)
        sincos(2.0 * M_PI * tg.t[t].fd_prt * j, &s, &c);
    else
        sincos((double)(j - g.P) * tg.t[t].dphi, &s, &c);
    tab[i] = d2{c, s};
}

// S4 + S4.1 on the device, laid out so that everything shared is loaded once: a wave owns one
// fast-time strip of SYNTH_NS samples n of one channel c (both wave-uniform, so the tx_pulse
// samples and the channel phasors are scalar loads), a lane owns the pulse pair (m, m + 1), and
// each target's two Doppler phasors are read once per strip, not once per sample. The pair is one
// Philox4x32-10 block (P is even, so flat indices 2q, 2q + 1 of the [C][N][P] order): the first
// sample takes words 0-1, the second 2-3 (oracle/philox.py documents the stream). Per sample the
// targets are summed in order (fsf:51-78), then the Box-Muller noise is added (fsf:80-88).
#define SYNTH_NS 8   // 4: same time, 16: +10 % (profiles/r06q_synth_ab.txt)
template <class T>
__global__ __launch_bounds__(RSP_THREADS) void k_synth(Geometry g, const double* __restrict__ tx, SynthTargets tg,
                                                          int nt, const d2* __restrict__ tab, int frame_idx,
                                                          uint64_t seed, double nscale, cx<T>* __restrict__ cube) {
    const int lane = threadIdx.x & 63;
    const int n0 = __builtin_amdgcn_readfirstlane((int)(blockIdx.y * (RSP_THREADS / 64) + (threadIdx.x >> 6)) * SYNTH_NS);
    if (n0 >= g.N) return;   // the whole wave
    const int c = blockIdx.z;
    const int m = 2 * ((int)blockIdx.x * 64 + lane);
    const bool act = m < g.P;
    const int per = g.P + g.C;
    double re[SYNTH_NS][2], im[SYNTH_NS][2];
#pragma unroll
    for (int u = 0; u < SYNTH_NS; ++u) re[u][0] = re[u][1] = im[u][0] = im[u][1] = 0.0;
    for (int t = 0; t < nt; ++t) {
        const int ds = tg.t[t].delay;
        if (!(ds > 0 && ds < g.N) || n0 + SYNTH_NS - 1 < ds) continue;
        const d2 d0 = act ? tab[t * per + m] : d2{}, d1 = act ? tab[t * per + m + 1] : d2{};
        const d2 cp = tab[t * per + g.P + c];
        const double amp = tg.t[t].amp;
#pragma unroll
        for (int u = 0; u < SYNTH_NS; ++u) {
            const int n = n0 + u;
            if (n < g.N && n >= ds) {
                const double tr = tx[2 * (n - ds)], ti = tx[2 * (n - ds) + 1];
                double er = amp * (tr * d0.x - ti * d0.y);   // amplitude * base * doppler
                double ei = amp * (tr * d0.y + ti * d0.x);
                re[u][0] += er * cp.x - ei * cp.y;
                im[u][0] += er * cp.y + ei * cp.x;
                er = amp * (tr * d1.x - ti * d1.y);
                ei = amp * (tr * d1.y + ti * d1.x);
                re[u][1] += er * cp.x - ei * cp.y;
                im[u][1] += er * cp.y + ei * cp.x;
            }
        }
    }
    if (!act) return;
#pragma unroll
    for (int u = 0; u < SYNTH_NS; ++u) {
        const int n = n0 + u;
        if (n >= g.N) break;
        const uint64_t q = ((uint64_t)c * g.N + n) * (uint64_t)(g.P >> 1) + (uint64_t)(m >> 1);   // flat index / 2
        uint32_t ctr[4] = {(uint32_t)q, (uint32_t)(q >> 32), (uint32_t)frame_idx, 0x52535020u};
        rsp_philox10(ctr, (uint32_t)seed, (uint32_t)(seed >> 32));
        cx<T>* dst = cube + (size_t)c * g.cpitch + (size_t)n * g.P + m;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const uint32_t xa = h ? ctr[2] : ctr[0];
            const uint32_t xb = h ? ctr[3] : ctr[1];
            const double ua = ((double)xa + 0.5) * 2.3283064365386963e-10;
            const double ub = ((double)xb + 0.5) * 2.3283064365386963e-10;
            const double rr = sqrt(-2.0 * rsp_nm_log(ua));
            double sb, cb;
            rsp_nm_sincos2pi(ub, &sb, &cb);   // sincos(2 pi ub)
            dst[h] = cx<T>{(T)(re[u][h] + rr * cb * nscale), (T)(im[u][h] + rr * sb * nscale)};
        }
    }
}

// ======================================================================================
// Detection lists -> pinned host memory (the queue's read-back, after K3)
// ======================================================================================
// Frame f = blockIdx.x: record 0 (the count) and the first min(count, dcap, hcap) detections
// from the device list (stride dcap + 1 records) into the mapped host list (stride hcap + 1), so
// only the records that exist cross PCIe, whatever the count (a fixed-size async copy moved the
// first 512 and left the rest to a synchronous tail copy).
__global__ __launch_bounds__(RSP_THREADS) void k_dets_to_host(const DevDet* __restrict__ dets, int dcap,
                                                             DevDet* __restrict__ host, int hcap) {
    const int f = blockIdx.x;
    const u32x4* src = reinterpret_cast<const u32x4*>(dets + (size_t)f * (dcap + 1));
    u32x4* dst = reinterpret_cast<u32x4*>(host + (size_t)f * (hcap + 1));
    const int cnt = *reinterpret_cast<const int*>(src);
    const int n = 1 + min(cnt, min(dcap, hcap));   // records, the count record included
    constexpr int U = sizeof(DevDet) / 16;        // 16-B units per record
    for (int e = threadIdx.x; e < n * U; e += RSP_THREADS) dst[e] = src[e];
}

}  // namespace

hipError_t launch_dets_to_host(const void* dets, int dcap, void* host, int hcap, int nf, hipStream_t s) {
    static_assert(sizeof(DevDet) % 16 == 0, "16-B units");
    hipLaunchKernelGGL(k_dets_to_host, dim3(nf), dim3(RSP_THREADS), 0, s, static_cast<const DevDet*>(dets), dcap,
                       static_cast<DevDet*>(host), hcap);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------------------
// Dynamic LDS above 64 KiB must be opted in per kernel (gfx950 has 160 KiB per CU).
template <class K>
static hipError_t allow_lds(K kernel, size_t bytes) {
    if (bytes <= 64 * 1024) return hipSuccess;
    return hipFuncSetAttribute(reinterpret_cast<const void*>(kernel), hipFuncAttributeMaxDynamicSharedMemorySize,
                               (int)bytes);
}

static size_t cplx_bytes(const Geometry& g) { return g.prec == RSP_PREC_F64 ? 16 : 8; }
static int k1_tpw(const Geometry& g) {
    const int cp = g.C <= 8 ? 8 : (g.C <= 16 ? 16 : 32), bmax = g.B <= 4 ? 4 : (g.B <= 8 ? 8 : 16);
    const int nj = cp / 4, mb = bmax <= 8 ? 1 : 2;
    return (16 / nj) / mb > 0 ? (16 / nj) / mb : 1;
}
// tile buffers x 2 | FFT twiddles (<= P) | two MFMA row blocks' Atab when B > 8 (k1p_dbf_mtd ALDS)
static size_t k1p_lds(const Geometry& g) {
    const int cp = g.C <= 8 ? 8 : (g.C <= 16 ? 16 : 32);
    return ((size_t)2 * g.B * g.NT * g.Ppad + g.P) * cplx_bytes(g) +
           (g.B > 8 ? (size_t)2 * (cp / 4) * 2 * 64 * (cplx_bytes(g) / 2) : 0);
}

// sub-tiles per wave of the persistent K1 (one load round per tile): TPW, or 2 TPW
static int k1p_tpw(const Geometry& g) {
    const int pt = g.prec == RSP_PREC_F64 ? 16 : 32;   // pulses per MFMA sub-tile
    const int need = (g.NT * (g.P / pt) + (K1_THREADS / 64) - 1) / (K1_THREADS / 64);
    return need <= k1_tpw(g) ? k1_tpw(g) : (need <= 2 * k1_tpw(g) ? 2 * k1_tpw(g) : 0);
}

// sub-tiles per wave of the factored-DFT K1 (one load round per tile): ceil(sub-tiles / 8) <= 4
static int k1q_tpw(const Geometry& g) {
    const int pt = g.prec == RSP_PREC_F64 ? 16 : 32;
    const int need = (g.NT * ((g.P + pt - 1) / pt) + (K1_THREADS / 64) - 1) / (K1_THREADS / 64);
    return need <= 4 ? need : 0;
}
static size_t k1q_lds(const Geometry& g) {   // tile | twQ | W_P^i | Atab (MB x NJ x 2 x 64 <= 1024 reals: CP <= 16)
    return ((size_t)g.B * g.NT * g.Ppad + g.twq_elems + g.P) * cplx_bytes(g) + (size_t)1024 * (cplx_bytes(g) / 2);
}
static bool k1q_fits(const Geometry& g) {
    return !g.pow2P && g.rqQ > 0 && k1q_tpw(g) > 0 && k1q_lds(g) <= 160 * 1024 && g.ncu > 0 && !g.k1_tiled;
}

bool k1_persistent_fits(const Geometry& g) {
    const int pts = g.prec == RSP_PREC_F64 ? 8 : 16;   // FFT points per thread (k1p_pts)
    return g.pow2P && g.logP >= 6 && g.logP <= 8 && k1p_tpw(g) > 0 && k1p_lds(g) <= 160 * 1024 &&
           g.B * g.NT * g.P <= pts * K1_THREADS && g.ncu > 0 && !g.k1_tiled;
}

template <class T, int BMAX, int CP>
static hipError_t launch_k1_t(const Geometry& g, const DevConsts& k, const FramePtrs& fp, int nf, int mode,
                              hipStream_t s) {
    if (mode == 3 && k1_persistent_fits(g)) {
        // one FFT size per instantiation keeps the prefetch registers + FFT under 256 VGPRs
        const size_t ldsp = k1p_lds(g);
        const int grid = std::min(g.ncu, nf * g.ntiles);
        constexpr int NJ = CP / 4, MB = BMAX <= 8 ? 1 : 2, TPW = (16 / NJ) / MB > 0 ? (16 / NJ) / MB : 1;
        const bool twice = k1p_tpw(g) == 2 * TPW;
#define K1P_LAUNCH(LGP, TW)                                                                                      \
    do {                                                                                                         \
        hipError_t e = allow_lds(k1p_dbf_mtd<T, BMAX, CP, LGP, TW>, ldsp);                                       \
        if (e != hipSuccess) return e;                                                                           \
        hipLaunchKernelGGL((k1p_dbf_mtd<T, BMAX, CP, LGP, TW>), dim3(grid), dim3(K1_THREADS), ldsp, s, g, k, fp, nf); \
        return hipGetLastError();                                                                                \
    } while (0)
        // 2 TPW sub-tiles per wave only where their loads stay within 16 16-B registers per lane
        // and 4 sub-tiles (x4: 2 x 8 channels); otherwise (no instantiation: it would spill) the
        // tiled kernel below
        constexpr bool TWICE_OK = 2 * TPW * NJ <= 16 && 2 * TPW <= 4;
        if (!twice || TWICE_OK) {
            switch (g.logP) {
                case 6: if constexpr (TWICE_OK) { if (twice) K1P_LAUNCH(6, 2 * TPW); } K1P_LAUNCH(6, TPW);
                case 7: if constexpr (TWICE_OK) { if (twice) K1P_LAUNCH(7, 2 * TPW); } K1P_LAUNCH(7, TPW);
                case 8: if constexpr (TWICE_OK) { if (twice) K1P_LAUNCH(8, 2 * TPW); } K1P_LAUNCH(8, TPW);
                default: break;
            }
        }
#undef K1P_LAUNCH
    }
    // the persistent factored-DFT K1 for C <= 16 when one load round of at most 16 16-B cube loads
    // per lane covers a tile (register budget: no scratch); otherwise the tiled kernel
    if constexpr (CP <= 16) {
        constexpr int NJ = CP / 4;
        if (mode == 3 && k1q_fits(g) && k1q_tpw(g) * NJ <= 16) {
            const size_t ldsq = k1q_lds(g);
            const int grid = std::min(g.ncu, nf * g.ntiles);
            hipError_t e;
#define K1Q_LAUNCH(TW)                                                                                            \
    do {                                                                                                          \
        if ((e = allow_lds(k1q_dbf_mtd<T, BMAX, CP, TW>, ldsq)) != hipSuccess) return e;                           \
        hipLaunchKernelGGL((k1q_dbf_mtd<T, BMAX, CP, TW>), dim3(grid), dim3(K1_THREADS), ldsq, s, g, k, fp, nf); \
    } while (0)
            switch (k1q_tpw(g)) {
                case 1: K1Q_LAUNCH(1); break;
                case 2: K1Q_LAUNCH(2); break;
                case 3: K1Q_LAUNCH(3); break;
                default: if constexpr (NJ <= 4) K1Q_LAUNCH(4); break;
            }
#undef K1Q_LAUNCH
            return hipGetLastError();
        }
    }
    const bool rq = (mode & 2) && !g.pow2P && g.rqQ > 0;
    const size_t lds = ((size_t)g.B * g.NT * g.Ppad + g.P + (rq ? g.twq_elems : 0)) * sizeof(cx<T>);
    hipError_t e;
    if (rq) {
        if ((e = allow_lds(k1_dbf_mtd<T, BMAX, CP, true>, lds)) != hipSuccess) return e;
        hipLaunchKernelGGL((k1_dbf_mtd<T, BMAX, CP, true>), dim3(g.ntiles, nf), dim3(K1_THREADS), lds, s, g, k, fp, mode);
    } else {
        if ((e = allow_lds(k1_dbf_mtd<T, BMAX, CP, false>, lds)) != hipSuccess) return e;
        hipLaunchKernelGGL((k1_dbf_mtd<T, BMAX, CP, false>), dim3(g.ntiles, nf), dim3(K1_THREADS), lds, s, g, k, fp, mode);
    }
    return hipGetLastError();
}

template <class T, int BMAX>
static hipError_t launch_k1_b(const Geometry& g, const DevConsts& k, const FramePtrs& fp, int nf, int mode,
                              hipStream_t s) {
    if (g.C <= 8) return launch_k1_t<T, BMAX, 8>(g, k, fp, nf, mode, s);
    if (g.C <= 16) return launch_k1_t<T, BMAX, 16>(g, k, fp, nf, mode, s);
    return launch_k1_t<T, BMAX, 32>(g, k, fp, nf, mode, s);
}

template <class T>
static hipError_t launch_k1_p(const Geometry& g, const DevConsts& k, const FramePtrs& fp, int nf, int mode,
                              hipStream_t s) {
    if (g.B <= 4) return launch_k1_b<T, 4>(g, k, fp, nf, mode, s);
    if (g.B <= 8) return launch_k1_b<T, 8>(g, k, fp, nf, mode, s);
    return launch_k1_b<T, 16>(g, k, fp, nf, mode, s);
}

hipError_t launch_k1(const Geometry& g, const DevConsts& k, const FramePtrs& fp, int nf, int mode, hipStream_t s) {
    return g.prec == RSP_PREC_F64 ? launch_k1_p<double>(g, k, fp, nf, mode, s)
                                  : launch_k1_p<float>(g, k, fp, nf, mode, s);
}

template <class T>
static hipError_t launch_k2_p(const Geometry& g, const DevConsts& k, const FramePtrs& fp, int nf, int rows,
                              hipStream_t s) {
    // workgroups sized for the 2560-point block (complex double): 4 per CU, the row's LDS alone
    const bool w4 = g.k2_pts != RSP_K2_POINTS;
    const size_t lds = w4 ? (size_t)g.k2_pts * sizeof(cx<T>)
                          : (size_t)(k2_lds_data(g.k2_pts, k2_sh<T>()) + k2_tw_lds_max()) * sizeof(cx<T>);
    hipError_t e = w4 ? allow_lds(k2_pc<T, 4>, lds) : allow_lds(k2_pc<T, 2>, lds);
    if (e != hipSuccess) return e;
    if (g.nwg_k2 > 0) {
        if (w4)
            hipLaunchKernelGGL((k2_pc<T, 4>), dim3(g.nwg_k2, nf), dim3(K2_THREADS), lds, s, g, k, fp, rows);
        else
            hipLaunchKernelGGL((k2_pc<T, 2>), dim3(g.nwg_k2, nf), dim3(K2_THREADS), lds, s, g, k, fp, rows);
    }
    return hipGetLastError();
}

// Streaming copy (rsp_hbm_copy_probe): CU16 x 16 B per lane, all loads in flight before the
// stores, one chunk per workgroup.
#define RSP_COPY_U 4    // 16-B loads per lane in flight; non-temporal both ways (6.2-6.5 TB/s at 0.25-1 GiB, 5.7-5.9 plain)
__global__ __launch_bounds__(256) void k_stream_copy(const u32x4* __restrict__ in, u32x4* __restrict__ out, size_t n16) {
    const size_t base = (size_t)blockIdx.x * (256 * RSP_COPY_U) + threadIdx.x;
    u32x4 v[RSP_COPY_U];
#pragma unroll
    for (int u = 0; u < RSP_COPY_U; ++u)
        if (base + u * 256 < n16) v[u] = __builtin_nontemporal_load(in + base + u * 256);
#pragma unroll
    for (int u = 0; u < RSP_COPY_U; ++u)
        if (base + u * 256 < n16) __builtin_nontemporal_store(v[u], out + base + u * 256);
}

hipError_t launch_stream_copy(const void* in, void* out, size_t n16, int, hipStream_t s) {
    hipLaunchKernelGGL(k_stream_copy, dim3((unsigned)((n16 + 256 * RSP_COPY_U - 1) / (256 * RSP_COPY_U))), dim3(256), 0, s,
                       static_cast<const u32x4*>(in), static_cast<u32x4*>(out), n16);
    return hipGetLastError();
}

hipError_t launch_k2(const Geometry& g, const DevConsts& k, const FramePtrs& fp, int nf, int rows, hipStream_t s) {
    return g.prec == RSP_PREC_F64 ? launch_k2_p<double>(g, k, fp, nf, rows, s)
                                  : launch_k2_p<float>(g, k, fp, nf, rows, s);
}

template <class T>
static hipError_t launch_k3_p(const Geometry& g, const DevConsts& k, const FramePtrs& fp, int nf, hipStream_t s) {
    const size_t lds = (size_t)g.cfar_rows * g.cfar_W * sizeof(T) + (K3_QCAP + 4) * sizeof(int);
    const dim3 grid(k3_ntiles(g) * g.cfar_nband * (g.B - 1) * nf);   // 1-D; k3_cfar remaps it XCD-aware
    hipError_t e;
    const bool ref = k3_fast_params(g);   // the reference's cfar_params (v8:45-46); the plan sized the tile for it
    if (ref && g.cfar_RT == 64) {
        if ((e = allow_lds(k3_cfar<T, 5, 5, 10, 10, 64>, lds)) != hipSuccess) return e;
        hipLaunchKernelGGL((k3_cfar<T, 5, 5, 10, 10, 64>), grid, dim3(RSP_THREADS), lds, s, g, k, fp);
    } else if (ref && g.cfar_RT == 32) {
        if ((e = allow_lds(k3_cfar<T, 5, 5, 10, 10, 32>, lds)) != hipSuccess) return e;
        hipLaunchKernelGGL((k3_cfar<T, 5, 5, 10, 10, 32>), grid, dim3(RSP_THREADS), lds, s, g, k, fp);
    } else {
        if ((e = allow_lds(k3_cfar<T, 0, 0, 0, 0, 0>, lds)) != hipSuccess) return e;
        hipLaunchKernelGGL((k3_cfar<T, 0, 0, 0, 0, 0>), grid, dim3(RSP_THREADS), lds, s, g, k, fp);
    }
    return hipGetLastError();
}

hipError_t launch_k3(const Geometry& g, const DevConsts& k, const FramePtrs& fp, int nf, hipStream_t s) {
    if (g.B < 2 || g.G - 2 * (g.refR + g.guardR) <= 0) return hipSuccess;
    return g.prec == RSP_PREC_F64 ? launch_k3_p<double>(g, k, fp, nf, s) : launch_k3_p<float>(g, k, fp, nf, s);
}

template <class T, int LGP>
static hipError_t launch_mtd_t(const Geometry& g, const DevConsts& k, const void* pc, void* rdm, hipStream_t s) {
    const size_t lds = ((size_t)16 * g.Ppad + g.P) * sizeof(cx<T>);
    hipError_t e = allow_lds(k_mtd_cols<T, LGP>, lds);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL((k_mtd_cols<T, LGP>), dim3((g.G + 15) / 16, g.B), dim3(RSP_THREADS), lds, s, g, k,
                       static_cast<const cx<T>*>(pc), static_cast<cx<T>*>(rdm));
    return hipGetLastError();
}

template <class T>
static hipError_t launch_mtd_p(const Geometry& g, const DevConsts& k, const void* pc, void* rdm, hipStream_t s) {
    switch (g.pow2P ? g.logP : 0) {
        case 4: return launch_mtd_t<T, 4>(g, k, pc, rdm, s);
        case 5: return launch_mtd_t<T, 5>(g, k, pc, rdm, s);
        case 6: return launch_mtd_t<T, 6>(g, k, pc, rdm, s);
        case 7: return launch_mtd_t<T, 7>(g, k, pc, rdm, s);
        case 8: return launch_mtd_t<T, 8>(g, k, pc, rdm, s);
        case 9: return launch_mtd_t<T, 9>(g, k, pc, rdm, s);
        default: return launch_mtd_t<T, 0>(g, k, pc, rdm, s);
    }
}

hipError_t launch_mtd_cols(const Geometry& g, const DevConsts& k, const void* pc, void* rdm, hipStream_t s) {
    return g.prec == RSP_PREC_F64 ? launch_mtd_p<double>(g, k, pc, rdm, s) : launch_mtd_p<float>(g, k, pc, rdm, s);
}

hipError_t launch_synth(const Geometry& g, const double* tx, const SynthTargets& tg, int nt, void* tab, int frame_idx,
                        uint64_t seed, double nscale, void* cube, hipStream_t s) {
    if (g.P & 1) return hipErrorInvalidValue;   // pulse pairs are Philox pairs; plans reject odd P at creation
    if (nt > 0)
        hipLaunchKernelGGL(k_synth_tab, dim3((nt * (g.P + g.C) + RSP_THREADS - 1) / RSP_THREADS), dim3(RSP_THREADS), 0, s,
                           g, tg, nt, static_cast<d2*>(tab));
    constexpr int rows = SYNTH_NS * (RSP_THREADS / 64);   // fast-time samples per workgroup
    const dim3 grid((g.P / 2 + 63) / 64, (g.N + rows - 1) / rows, g.C);
    if (g.prec == RSP_PREC_F64)
        hipLaunchKernelGGL(k_synth<double>, grid, dim3(RSP_THREADS), 0, s, g, tx, tg, nt, static_cast<const d2*>(tab),
                           frame_idx, seed, nscale, static_cast<d2*>(cube));
    else
        hipLaunchKernelGGL(k_synth<float>, grid, dim3(RSP_THREADS), 0, s, g, tx, tg, nt, static_cast<const d2*>(tab),
                           frame_idx, seed, nscale, static_cast<f2*>(cube));
    return hipGetLastError();
}
