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
//                 fused into the output store -> RDM [B][P][G].
//   k3_cfar     : |RDM| adjacent-beam sum (fsf:184-187), cross GOCA-CFAR (fsf:192-213),
//                 atomic compaction (fsf:215-221) and S9 spline/monopulse estimation
//                 (fsf:237-290) of each detection.
//   k_mtd_cols  : MTD over pulses of a pulse-compressed cube (stage-2 path).
//   k_synth     : S4 echo synthesis + S4.1 Philox noise (fsf:45-88) on the device.
#include "rsp_internal.h"
#include <math.h>

namespace {

__device__ __forceinline__ float2 cmul(float2 a, float2 b) {
    return make_float2(a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x);
}
__device__ __forceinline__ float2 cadd(float2 a, float2 b) { return make_float2(a.x + b.x, a.y + b.y); }
__device__ __forceinline__ float2 csub(float2 a, float2 b) { return make_float2(a.x - b.x, a.y - b.y); }

// ---- complex values as 2-wide float vectors ---------------------------------------------
// The FFT core keeps every complex value in one ext_vector pair, so complex adds are single
// v_pk_add_f32 and complex products two packed ops, without the register shuffles the
// compiler's SLP packing of struct float2 code produces.
typedef float f2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ f2 tof2(float2 a) { return f2{a.x, a.y}; }
__device__ __forceinline__ float2 fromf2(f2 a) { return make_float2(a.x, a.y); }

// Raw buffer resources (SRSRC): 32-bit byte offsets and hardware range checking.  An offset at
// or past num_records reads 0 / drops the store, so masked lanes need no branch or select.
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
#define RSP_OOB 0x80000000u   // > any buffer this library makes (plans are validated < 2 GB/frame)
__device__ __forceinline__ __amdgpu_buffer_rsrc_t buf_rsrc(const void* p, unsigned bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, (int)bytes, 0x00020000);
}
__device__ __forceinline__ f2 buf_ld_f2(__amdgpu_buffer_rsrc_t r, unsigned off) {
    const u32x2 v = __builtin_amdgcn_raw_buffer_load_b64(r, (int)off, 0, 0);
    return f2{__uint_as_float(v.x), __uint_as_float(v.y)};
}
#ifndef RSP_ST_AUX
#define RSP_ST_AUX 0
#endif
template <int AUX = 0>
__device__ __forceinline__ void buf_st_f2(__amdgpu_buffer_rsrc_t r, unsigned off, f2 x) {
    __builtin_amdgcn_raw_buffer_store_b64(u32x2{__float_as_uint(x.x), __float_as_uint(x.y)}, r, (int)off, 0, AUX);
}
__device__ __forceinline__ void buf_st_f1(__amdgpu_buffer_rsrc_t r, unsigned off, float x) {
    __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(x), r, (int)off, 0, 0);
}
// |x| with the hardware square root (v_sqrt_f32, 1 ulp) instead of the correctly rounded
// sequence (~15 VALU): the magnitude map feeds threshold tests at fp32 noise level anyway
__device__ __forceinline__ float fast_abs(f2 x) { return __builtin_amdgcn_sqrtf(x.x * x.x + x.y * x.y); }
__device__ __forceinline__ f2 vmul(f2 a, f2 b) { return a.xx * b + a.yy * f2{-b.y, b.x}; }
template <bool INV>
__device__ __forceinline__ f2 vrot(f2 a) {   // * (-i) forward, * (+i) inverse
    return INV ? a.yx * f2{-1.f, 1.f} : a.yx * f2{1.f, -1.f};
}
template <bool INV>
__device__ __forceinline__ f2 vtw(float c, float s) { return f2{c, INV ? s : -s}; }   // exp(-+ i theta)

// ---- radix-R DFT kernels in registers -------------------------------------------------
template <int R, bool INV> struct Dft;
template <bool INV> struct Dft<2, INV> {
    static __device__ __forceinline__ void run(f2* a) {
        const f2 t = a[0];
        a[0] = t + a[1];
        a[1] = t - a[1];
    }
};
template <bool INV> struct Dft<4, INV> {
    static __device__ __forceinline__ void run(f2* a) {
        const f2 t0 = a[0] + a[2], t1 = a[0] - a[2];
        const f2 t2 = a[1] + a[3], t3 = vrot<INV>(a[1] - a[3]);
        a[0] = t0 + t2;
        a[2] = t0 - t2;
        a[1] = t1 + t3;
        a[3] = t1 - t3;
    }
};
template <bool INV> struct Dft<8, INV> {
    static __device__ __forceinline__ void run(f2* a) {
        f2 e[4] = {a[0], a[2], a[4], a[6]};
        f2 o[4] = {a[1], a[3], a[5], a[7]};
        Dft<4, INV>::run(e);
        Dft<4, INV>::run(o);
        const float r = 0.70710678118654752f;
        o[1] = vmul(o[1], vtw<INV>(r, r));
        o[2] = vrot<INV>(o[2]);
        o[3] = vmul(o[3], vtw<INV>(-r, r));
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            a[k] = e[k] + o[k];
            a[k + 4] = e[k] - o[k];
        }
    }
};
template <bool INV> struct Dft<16, INV> {
    static __device__ __forceinline__ void run(f2* a) {
        f2 e[8], o[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            e[k] = a[2 * k];
            o[k] = a[2 * k + 1];
        }
        Dft<8, INV>::run(e);
        Dft<8, INV>::run(o);
        const float c1 = 0.92387953251128674f, s1 = 0.38268343236508977f, r = 0.70710678118654752f;
        o[1] = vmul(o[1], vtw<INV>(c1, s1));
        o[2] = vmul(o[2], vtw<INV>(r, r));
        o[3] = vmul(o[3], vtw<INV>(s1, c1));
        o[4] = vrot<INV>(o[4]);
        o[5] = vmul(o[5], vtw<INV>(-s1, c1));
        o[6] = vmul(o[6], vtw<INV>(-r, r));
        o[7] = vmul(o[7], vtw<INV>(-c1, s1));
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            a[k] = e[k] + o[k];
            a[k + 8] = e[k] - o[k];
        }
    }
};

template <bool INV> struct Dft<5, INV> {   // X1 = m1 + rot(n1), X4 = m1 - rot(n1), X2 = m2 + rot(n2), X3 = m2 - rot(n2)
    static __device__ __forceinline__ void run(f2* a) {
        const float c1 = 0.30901699437494742f, c2 = -0.80901699437494742f;   // cos(2 pi / 5), cos(4 pi / 5)
        const float s1 = 0.95105651629515357f, s2 = 0.58778525229247313f;    // sin(2 pi / 5), sin(4 pi / 5)
        const f2 t1 = a[1] + a[4], t2 = a[2] + a[3], t3 = a[1] - a[4], t4 = a[2] - a[3];
        const f2 m1 = a[0] + c1 * t1 + c2 * t2, m2 = a[0] + c2 * t1 + c1 * t2;
        const f2 n1 = vrot<INV>(s1 * t3 + s2 * t4), n2 = vrot<INV>(s2 * t3 - s1 * t4);
        a[0] = a[0] + t1 + t2;
        a[1] = m1 + n1;
        a[4] = m1 - n1;
        a[2] = m2 + n2;
        a[3] = m2 - n2;
    }
};
template <bool INV> struct Dft<10, INV> {   // 2 x 5 (even / odd halves, W_10^k on the odd)
    static __device__ __forceinline__ void run(f2* a) {
        f2 e[5], o[5];
#pragma unroll
        for (int k = 0; k < 5; ++k) {
            e[k] = a[2 * k];
            o[k] = a[2 * k + 1];
        }
        Dft<5, INV>::run(e);
        Dft<5, INV>::run(o);
        const float c1 = 0.80901699437494742f, s1 = 0.58778525229247313f;   // W_10^1
        const float c2 = 0.30901699437494742f, s2 = 0.95105651629515357f;   // W_10^2
        o[1] = vmul(o[1], vtw<INV>(c1, s1));
        o[2] = vmul(o[2], vtw<INV>(c2, s2));
        o[3] = vmul(o[3], vtw<INV>(-c2, s2));
        o[4] = vmul(o[4], vtw<INV>(-c1, s1));
#pragma unroll
        for (int k = 0; k < 5; ++k) {
            a[k] = e[k] + o[k];
            a[k + 5] = e[k] - o[k];
        }
    }
};

constexpr int clog2(int x) { return x <= 1 ? 0 : 1 + clog2(x >> 1); }

// LDS index inside a row: SH > 0 inserts one complex every 2^SH to break power-of-two
// strides (tools/lds_conflicts.py models the gfx950 bank rules for each pass).
template <int SH>
__device__ __forceinline__ int lidx(int i) { return SH ? i + (i >> SH) : i; }

// Store policies for the Stockham pass output.  put(idx, row, o, loff, x): idx = t * R + r for
// butterfly t / element r of this thread (a constant after unrolling), row, natural position
// o, and the padded LDS offset loff of (row, o).
struct StoreLds {
    float2* buf;
    __device__ __forceinline__ void put(int, int, int, int loff, f2 x) const { buf[loff] = fromf2(x); }
};

// Last forward pass of the overlap-save FFT: multiply by the block filter spectrum H (1/M
// folded in), prefetched into registers at kernel start (h[t * R + r] for this thread's outputs).
template <int NH>
struct StoreLdsH {
    float2* buf;
    const f2 (&h)[NH];
    __device__ __forceinline__ void put(int idx, int, int, int loff, f2 x) const { buf[loff] = fromf2(vmul(x, h[idx])); }
};

// Twiddles w[r] = W_{Ns R}^{k r}, r = 1..R-1, of one butterfly (conjugated for the inverse)
// from this pass's table row k: CMP = false: full rows [k][r-1] (R-1 loads); CMP = true:
// compact rows [k][i] = W^(k 2^i) (lgR loads), the other powers formed as products of at
// most lgR - 1 of them.
template <int R, bool INV, bool CMP>
__device__ __forceinline__ void load_tw(const float2* twk, f2 (&w)[R]) {
    if constexpr (!CMP) {
#pragma unroll
        for (int r = 1; r < R; ++r) {
            const float2 t = twk[r - 1];
            w[r] = f2{t.x, INV ? -t.y : t.y};
        }
    } else {
        constexpr int lgR = clog2(R - 1) + 1;   // bases W^(k 2^i), 2^i < R (= log2 R for powers of two)
        f2 b[lgR];
#pragma unroll
        for (int i = 0; i < lgR; ++i) {
            const float2 t = twk[i];
            b[i] = f2{t.x, INV ? -t.y : t.y};
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
constexpr int rad_bits_p(int m, int q, bool rev) { return rev ? rad_bits(m, n_passes(m) - 1 - q) : rad_bits(m, q); }

// Offset of pass q's twiddle table inside the concatenated per-pass tables of a 2^LG FFT:
// pass i >= 1 owns Ns_i rows of tw_row(R_i) entries (pass 0: Ns = 1, no twiddles).  Must
// match build_pass_twiddles() in rsp_plan.cpp.
constexpr int tw_pass_off(int LG, int q, bool rev = false, bool cmp = false) {
    int off = 0, lgns = 0;
    for (int i = 0; i < q; ++i) {
        const int rb = rad_bits_p(LG, i, rev);
        if (i > 0) off += (1 << lgns) * tw_row(1 << rb, cmp);
        lgns += rb;
    }
    return off;
}
constexpr int tw_total(int LG, bool rev = false, bool cmp = false) { return tw_pass_off(LG, n_passes(LG), rev, cmp); }

// One Stockham radix-R pass (Govindaraju et al. formulation) over `nrows` rows of
// length L = 2^LGL held in LDS (row stride rs).  Ns = 2^LGNS = product of the earlier
// radices.  Reads stride L/R, twiddle W_{Ns R}^{(j mod Ns) r} (from this pass's table),
// radix-R DFT, writes positions expand(j, Ns, R) + r Ns.  In place: all reads, barrier,
// all writes, barrier.  Every size is a compile-time constant, so a pass is straight-line
// code and no address math is carried across passes.
// With power-of-two nb, Ns and pads every 2^SH, lidx(j + r nb) = lidx(j) + r nb + ((r nb) >> SH)
// and lidx(idxD + r Ns) = lidx(idxD) + r Ns + ((r Ns) >> SH): every LDS address of a butterfly
// is a per-thread base plus a compile-time offset (ds_read/ds_write immediate offsets).
template <int R, bool INV, int NB, int SH, int NTHR, int LGL, int LGNS, bool CMP = false>
__device__ __forceinline__ void sh_load(const float2* buf, int rs, int nrows, const float2* tw, f2 (&v)[NB][R]) {
    constexpr int lgR = clog2(R);
    constexpr int lgnb = LGL - lgR;
    constexpr int nb = 1 << lgnb;
    constexpr int Ns = 1 << LGNS;
    const int total = nb * nrows;
#pragma unroll
    for (int t = 0; t < NB; ++t) {
        const int beta = threadIdx.x + t * NTHR;
        if (beta < total) {
            const int row = beta >> lgnb, j = beta & (nb - 1);
            const int k = j & (Ns - 1);
            const float2* src = buf + row * rs + lidx<SH>(j);
            f2 w[R];
            if (LGNS > 0) load_tw<R, INV, CMP>(tw + k * tw_row(R, CMP), w);
#pragma unroll
            for (int r = 0; r < R; ++r) {
                f2 x = tof2(src[r * nb + (SH ? (r * nb) >> SH : 0)]);
                if (r > 0 && LGNS > 0) x = vmul(x, w[r]);
                v[t][r] = x;
            }
        }
    }
}

// Radix-R DFT of the loaded butterflies and the Stockham store (through policy st).
template <int R, bool INV, int NB, int SH, int NTHR, int LGL, int LGNS, class St>
__device__ __forceinline__ void sh_store(f2 (&v)[NB][R], int rs, int nrows, const St& st) {
    constexpr int lgR = clog2(R);
    constexpr int lgnb = LGL - lgR;
    constexpr int nb = 1 << lgnb;
    constexpr int Ns = 1 << LGNS;
    const int total = nb * nrows;
#pragma unroll
    for (int t = 0; t < NB; ++t) {
        const int beta = threadIdx.x + t * NTHR;
        if (beta < total) {
            const int row = beta >> lgnb, j = beta & (nb - 1);
            const int k = j & (Ns - 1);
            Dft<R, INV>::run(v[t]);
            const int idxD = ((j >> LGNS) << (LGNS + lgR)) + k;
            const int wbase = row * rs + lidx<SH>(idxD);
#pragma unroll
            for (int r = 0; r < R; ++r)
                st.put(t * R + r, row, idxD + r * Ns, wbase + r * Ns + (SH ? (r * Ns) >> SH : 0), v[t][r]);
        }
    }
}

template <int R, bool INV, int NB, int SH, int NTHR, int LGL, int LGNS, bool CMP, class St>
__device__ __forceinline__ void sh_pass(float2* buf, int rs, int nrows, const float2* tw, const St& st) {
    f2 v[NB][R];
    sh_load<R, INV, NB, SH, NTHR, LGL, LGNS, CMP>(buf, rs, nrows, tw, v);
    __syncthreads();
    sh_store<R, INV, NB, SH, NTHR, LGL, LGNS>(v, rs, nrows, st);
    __syncthreads();
}

// Passes Q..QEND-1 of a 2^LG-point FFT (radix order reversed if REV) over `nrows` rows;
// pass n_passes - 1 stores through `last`, the others through `mid`.  tw = this plan's
// concatenated tables.  PTS = complex points per thread (nrows * L / NTHR).
template <int LG, int Q, int QEND, int LGNS, int PTS, bool INV, bool REV, int SH, int NTHR, bool CMP, class StMid,
          class StLast>
__device__ __forceinline__ void fft_range(float2* buf, int rs, int nrows, const float2* tw, const StMid& mid,
                                          const StLast& last) {
    constexpr int NP = n_passes(LG);
    if constexpr (Q < QEND) {
        constexpr int RB = rad_bits_p(LG, Q, REV);
        constexpr int R = 1 << RB;
        constexpr int NB = (PTS + R - 1) / R;
        const float2* twq = tw + tw_pass_off(LG, Q, REV, CMP);
        if constexpr (Q == NP - 1)
            sh_pass<R, INV, NB, SH, NTHR, LG, LGNS, CMP>(buf, rs, nrows, twq, last);
        else
            sh_pass<R, INV, NB, SH, NTHR, LG, LGNS, CMP>(buf, rs, nrows, twq, mid);
        fft_range<LG, Q + 1, QEND, LGNS + RB, PTS, INV, REV, SH, NTHR, CMP>(buf, rs, nrows, tw, mid, last);
    }
}

// All passes of a 2^LG-point FFT over `nrows` rows; the last pass stores through `last`.
template <int LG, int Q, int LGNS, int PTS, bool INV, int SH, int NTHR, class StMid, class StLast>
__device__ __forceinline__ void fft_passes(float2* buf, int rs, int nrows, const float2* tw, const StMid& mid,
                                           const StLast& last) {
    fft_range<LG, Q, n_passes(LG), LGNS, PTS, INV, false, SH, NTHR, false>(buf, rs, nrows, tw, mid, last);
}

__device__ __forceinline__ int ilog2(int x) { return 31 - __clz(x); }

typedef float f32x4 __attribute__((ext_vector_type(4)));

// Diagnostic phase stamps (only when FramePtrs::trace is set: rsp_profile_stages with
// RSP_TRACE_FILE).  Stamp i of the linear workgroup id; 100 MHz constant clock.
__device__ __forceinline__ void trace_stamp(const FramePtrs& fp, int i) {
    if (fp.trace && threadIdx.x == 0) {
        const size_t wg = blockIdx.x + (size_t)gridDim.x * (blockIdx.y + (size_t)gridDim.y * blockIdx.z);
        fp.trace[wg * 4 + i] = __builtin_amdgcn_s_memrealtime();
    }
}

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
    const int lgNT = ilog2(g.NT);
    return (((size_t)b * g.ntiles + (np >> lgNT)) * g.P + v) * g.NT + (np & (g.NT - 1));
}

// ======================================================================================
// K1: DBF + MTD window + slow-time FFT + fftshift -> compacted rows
// ======================================================================================
#ifndef K1_THREADS
#define K1_THREADS 512
#endif
#define K1_SH 4   // LDS pad shift of the slow-time FFT rows (row stride P + P/16)

// Last slow-time FFT pass straight from registers to z with fftshift (fsf:135): column
// row = b NT + nl, frequency o -> Doppler cell v = (o + P/2) mod P.  16 lanes of a butterfly
// group write consecutive v of one column (64 B apart) and the next 16 lanes the neighbouring
// column (+8 B), so the lines fill within the workgroup.
struct StoreZ {
    __amdgpu_buffer_rsrc_t z; int lgNT, ntiles, tile, P, half;
    __device__ __forceinline__ void put(int, int row, int o, int, f2 x) const {
        const int b = row >> lgNT, nl = row & ((1 << lgNT) - 1);
        const int v = (o + half) & (P - 1);
        buf_st_f2<RSP_ST_AUX>(z, (unsigned)(((((b * ntiles + tile) * P + v) << lgNT) + nl)) * 8u, x);
    }
};

// Slow-time FFT of every (beam, sample) column in LDS for the runtime log2(P); the last pass
// stores through `last`.
template <class StLast>
__device__ __forceinline__ void k1_fft(int lgp, float2* Y, int Ppad, int ncols, const float2* twl, const StLast& last) {
    StoreLds st{Y};
    switch (lgp) {
        case 4: fft_passes<4, 0, 0, 16, false, K1_SH, K1_THREADS>(Y, Ppad, ncols, twl, st, last); break;
        case 5: fft_passes<5, 0, 0, 16, false, K1_SH, K1_THREADS>(Y, Ppad, ncols, twl, st, last); break;
        case 6: fft_passes<6, 0, 0, 16, false, K1_SH, K1_THREADS>(Y, Ppad, ncols, twl, st, last); break;
        case 7: fft_passes<7, 0, 0, 16, false, K1_SH, K1_THREADS>(Y, Ppad, ncols, twl, st, last); break;
        case 8: fft_passes<8, 0, 0, 16, false, K1_SH, K1_THREADS>(Y, Ppad, ncols, twl, st, last); break;
        default: fft_passes<9, 0, 0, 16, false, K1_SH, K1_THREADS>(Y, Ppad, ncols, twl, st, last); break;
    }
}

// BMAX = beams rounded up (4/8/16), CP = channels rounded up (8/16/32).  Weights are conj(W)
// laid out [CP][BMAX] in LDS, zero for padded beams/channels, so the DBF has no data-dependent
// branches: CP unconditional 8-B loads per (sample, pulse) all in flight together, then
// BMAX*CP complex FMAs whose weights are LDS broadcast reads.
template <int BMAX, int CP>
__global__ __launch_bounds__(K1_THREADS, 4) void k1_dbf_mtd(Geometry g, DevConsts k, FramePtrs fp, int mode) {
    extern __shared__ __attribute__((aligned(16))) float2 Y[];   // [B][NT][Ppad] | twiddles | W
    const int f = blockIdx.y, tile = blockIdx.x;
    const int B = g.B, C = g.C, P = g.P, NT = g.NT, Ppad = g.Ppad;
    trace_stamp(fp, 0);
    if (tile == 0 && threadIdx.x == 0 && fp.count[f]) *fp.count[f] = 0;   // K3's detection counter
    float2* twl = Y + B * NT * Ppad;
    const bool fft = (mode & 2) && g.pow2P;
    const int sh = fft ? K1_SH : 0;
    // twiddles: global loads issued first, LDS stores after the cube loads are in flight (the
    // barrier before the FFT orders them), so no load waits behind a barrier at kernel start
    constexpr int TWPRE = 2;
    float2 twv[TWPRE];
#pragma unroll
    for (int u = 0; u < TWPRE; ++u) {
        const int i = threadIdx.x + u * K1_THREADS;
        if (fft && i < g.twPp_elems) twv[u] = k.twPp[i];
    }
    const float2* __restrict__ x = fp.in[f];
    const size_t NP = (size_t)g.cpitch;   // channel stride
    if (mode & 1) {
        // ---- Phase A (MFMA): DBF (fsf:93-97) + MTD window (fsf:134) as a real GEMM on the
        // f32 matrix cores: D[16 x 16 pulses] += A[16 x 4 channels] * B[4 channels x 16 pulses],
        // rows = (Re, Im) x 8 beams, one MFMA per (channel group, Re/Im part, even/odd pulses).
        // Each lane loads 16 B = pulses (p, p+1) of one channel: B operand of two column blocks.
        constexpr int NJ = CP / 4, MB = BMAX <= 8 ? 1 : 2, TPW = (16 / NJ) / MB > 0 ? (16 / NJ) / MB : 1;
        const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, grp = lane >> 4, col = lane & 15;
        float are[MB][NJ], aim[MB][NJ];   // this lane's A operand: row lane&15, channel 4j + lane>>4
#pragma unroll
        for (int mb = 0; mb < MB; ++mb)
#pragma unroll
            for (int j = 0; j < NJ; ++j) {
                are[mb][j] = k.Atab[((mb * NJ + j) * 2 + 0) * 64 + lane];
                aim[mb][j] = k.Atab[((mb * NJ + j) * 2 + 1) * 64 + lane];
            }
        const int ptiles = (P + 31) >> 5;
        const int ntp = NT * ptiles;
        float* Yf = reinterpret_cast<float*>(Y);
        float sink = 0.f;
        // a wave takes TPW consecutive tiles (pulse tiles of the same sample first), so the
        // 1 KB pulse row of each (channel, sample) is fetched by one wave in one burst
        for (int t0 = wv * TPW; t0 < ntp; t0 += (K1_THREADS / 64) * TPW) {
            float4 xv[TPW][NJ];
            int nlv[TPW], pv[TPW];
#pragma unroll
            for (int u = 0; u < TPW; ++u) {      // every load of TPW tiles in flight together
                const int t = t0 + u;
                const int nl = t / ptiles;
                const int p = ((t - nl * ptiles) << 5) + 2 * col;
                const int np = tile * NT + nl;
                int n = -1;
                if (t < ntp && np < g.nU && p < P) {
                    n = used_sample(g, np);
                }
                nlv[u] = t < ntp ? nl : -1;
                pv[u] = p;
                if (g.dbg & 32) {   // ablation: same bytes, 1 KB-contiguous wave loads (timing only)
#pragma unroll
                    for (int j = 0; j < NJ; ++j) {
                        const int c = min(4 * j + (u & 3), C - 1);
                        const int pp = (2 * lane) % P;
                        xv[u][j] = n >= 0 ? *reinterpret_cast<const float4*>(x + (size_t)c * NP + (size_t)n * P + pp)
                                          : make_float4(0.f, 0.f, 0.f, 0.f);
                    }
                } else {
#pragma unroll
                    for (int j = 0; j < NJ; ++j) {
                        const int c = min(4 * j + grp, C - 1);   // padded channels carry zero weights
                        xv[u][j] = n >= 0 ? *reinterpret_cast<const float4*>(x + (size_t)c * NP + (size_t)n * P + p)
                                          : make_float4(0.f, 0.f, 0.f, 0.f);
                    }
                }
            }
            if (g.dbg & 128) {   // ablation (timing only): the cube loads alone, nothing computed
#pragma unroll
                for (int u = 0; u < TPW; ++u)
#pragma unroll
                    for (int j = 0; j < NJ; ++j) sink += xv[u][j].x + xv[u][j].y + xv[u][j].z + xv[u][j].w;
                continue;
            }
#pragma unroll
            for (int u = 0; u < TPW; ++u) {
                if (nlv[u] < 0) continue;
                f32x4 acc[MB][2];
#pragma unroll
                for (int mb = 0; mb < MB; ++mb) {
                    acc[mb][0] = f32x4{0.f, 0.f, 0.f, 0.f};
                    acc[mb][1] = acc[mb][0];
#pragma unroll
                    for (int j = 0; j < NJ; ++j) {
                        acc[mb][0] = __builtin_amdgcn_mfma_f32_16x16x4f32(are[mb][j], xv[u][j].x, acc[mb][0], 0, 0, 0);
                        acc[mb][0] = __builtin_amdgcn_mfma_f32_16x16x4f32(aim[mb][j], xv[u][j].y, acc[mb][0], 0, 0, 0);
                        acc[mb][1] = __builtin_amdgcn_mfma_f32_16x16x4f32(are[mb][j], xv[u][j].z, acc[mb][1], 0, 0, 0);
                        acc[mb][1] = __builtin_amdgcn_mfma_f32_16x16x4f32(aim[mb][j], xv[u][j].w, acc[mb][1], 0, 0, 0);
                    }
                }
                const int p = pv[u];
                if (p >= P) continue;
                float w0 = 1.f, w1 = 1.f;
                if (mode & 2) {
                    const float2 w01 = *reinterpret_cast<const float2*>(k.win + p);
                    w0 = w01.x;
                    w1 = w01.y;
                }
                const int i0 = sh ? p + (p >> K1_SH) : p, i1 = sh ? (p + 1) + ((p + 1) >> K1_SH) : p + 1;
#pragma unroll
                for (int mb = 0; mb < MB; ++mb)
#pragma unroll
                    for (int i = 0; i < 4; ++i) {   // D row m = 4*grp + i: beam mb*8 + (m & 7), part m >> 3
                        const int m = 4 * grp + i;
                        const int b = mb * 8 + (m & 7);
                        if (b < B && !(g.dbg & 1024)) {   // RSP_ABLATE=1024 skips the LDS writes
                            float* colp = Yf + 2 * (b * NT + nlv[u]) * Ppad + (m >> 3);
                            colp[2 * i0] = acc[mb][0][i] * w0;
                            colp[2 * i1] = acc[mb][1][i] * w1;
                        }
                    }
            }
        }
        if (g.dbg & 128) {
            if (sink == 1.2345e-30f) fp.z[f][threadIdx.x] = make_float2(sink, 0.f);   // keeps the loads
            return;
        }
    } else {
        // ---- transpose only (stage-2 path: input channels are the beams)
        const int items = NT * P;
        for (int it = threadIdx.x; it < items; it += K1_THREADS) {
            const int nl = it / P, p = it - nl * P;
            const int np = tile * NT + nl;
            int n = -1;
            if (np < g.nU) {
                n = used_sample(g, np);
            }
            const int ip = sh ? p + (p >> K1_SH) : p;
#pragma unroll
            for (int b = 0; b < BMAX; ++b) {
                if (b < B) {
                    float2 val = n >= 0 ? x[(size_t)b * NP + (size_t)n * P + p] : make_float2(0.f, 0.f);
                    if (mode & 2) {
                        val.x *= k.win[p];
                        val.y *= k.win[p];
                    }
                    Y[(b * NT + nl) * Ppad + ip] = val;
                }
            }
        }
    }
    if (fft) {
#pragma unroll
        for (int u = 0; u < TWPRE; ++u) {
            const int i = threadIdx.x + u * K1_THREADS;
            if (i < g.twPp_elems) twl[i] = twv[u];
        }
        for (int i = threadIdx.x + TWPRE * K1_THREADS; i < g.twPp_elems; i += K1_THREADS) twl[i] = k.twPp[i];
    }
    __syncthreads();
    trace_stamp(fp, 1);
    float2* __restrict__ z = fp.z[f];
    const int zslab = P * NT;   // contiguous [P][NT] slab per (b, tile)
    const int lgNT = ilog2(NT);
    if (!(mode & 2)) {
        for (int e = threadIdx.x; e < B * zslab; e += K1_THREADS) {
            const int b = e / zslab, rem = e - b * zslab;
            const int v = rem >> lgNT, nl = rem & (NT - 1);
            z[((size_t)b * g.ntiles + tile) * zslab + rem] = Y[(b * NT + nl) * Ppad + v];
        }
        return;
    }
    const int half = P >> 1;
    if (fft) {
        // ---- Phase B + C: P-point FFT of every (b, nl) column (fsf:135); the last pass applies
        // fftshift and stores the [P][NT] slabs from registers
        const StoreZ sz{buf_rsrc(z, (unsigned)B * g.ntiles * zslab * 8u), lgNT, g.ntiles, tile, P, half};
        if (!(g.dbg & 2)) k1_fft(g.logP, Y, Ppad, B * NT, twl, sz);   // RSP_ABLATE=2: no FFT, no store
        trace_stamp(fp, 2);
        if (fp.trace) trace_stamp(fp, 3);
    } else {
        // non power-of-two P: direct DFT straight to global (O(P^2) per column)
        for (int e = threadIdx.x; e < B * zslab; e += K1_THREADS) {
            const int b = e / zslab, rem = e - b * zslab;
            const int v = rem >> lgNT, nl = rem & (NT - 1);
            int kk = v - half;
            if (kk < 0) kk += P;
            const float2* col = Y + (b * NT + nl) * Ppad;
            float2 acc = make_float2(0.f, 0.f);
            int idx = 0;
            for (int p = 0; p < P; ++p) {
                acc = cadd(acc, cmul(col[p], k.twP[idx]));
                idx += kk;
                if (idx >= P) idx -= P;
            }
            z[((size_t)b * g.ntiles + tile) * zslab + rem] = acc;
        }
    }
}

// K1, persistent and software-pipelined (the default for power-of-two P when one load round
// covers a tile): one workgroup per CU walks the (frame, tile) list with two LDS tile buffers.
// While tile T's slow-time FFT runs out of one buffer and its last pass streams z to HBM, the
// cube loads of the workgroup's next tile are already in flight in registers; the DBF of that
// tile then fills the other buffer.  HBM reads and writes overlap instead of alternating
// round by round.  Same arithmetic as k1_dbf_mtd (mode 3).
template <int BMAX, int CP, int LGP>
__global__ __launch_bounds__(K1_THREADS, 1) void k1p_dbf_mtd(Geometry g, DevConsts k, FramePtrs fp, int nf) {
    extern __shared__ __attribute__((aligned(16))) float2 Y[];   // tile [B][NT][Ppad] (x2 if nbuf = 2) | twiddles
    const int B = g.B, C = g.C, P = g.P, NT = g.NT, Ppad = g.Ppad;
    const int nbuf = (g.dbg & 8192) ? 1 : 2;   // RSP_ABLATE=8192: one buffer (measured slower: 20.7k vs 21.2k frames/s)
    const int bufsz = B * NT * Ppad;
    float2* twl = Y + nbuf * bufsz;
    const int total = nf * g.ntiles;
    int T = blockIdx.x;
    if (T >= total) return;
    for (int i = threadIdx.x; i < g.twPp_elems; i += K1_THREADS) twl[i] = k.twPp[i];
    constexpr int NJ = CP / 4, MB = BMAX <= 8 ? 1 : 2, TPW = (16 / NJ) / MB > 0 ? (16 / NJ) / MB : 1;
    const int lane = threadIdx.x & 63, grp = lane >> 4, col = lane & 15;
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);   // wave-uniform: nlv[] and n are scalar
    float are[MB][NJ], aim[MB][NJ];
#pragma unroll
    for (int mb = 0; mb < MB; ++mb)
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
            are[mb][j] = k.Atab[((mb * NJ + j) * 2 + 0) * 64 + lane];
            aim[mb][j] = k.Atab[((mb * NJ + j) * 2 + 1) * 64 + lane];
        }
    // this lane's sub-tiles are the same for every tile: (sample nl, pulses p, p + 1) and their
    // window values (launch_k1 guarantees one round: NT * ptiles <= waves * TPW)
    const int ptiles = (P + 31) >> 5, ntp = NT * ptiles;
    int nlv[TPW], pv[TPW];
    float w0v[TPW], w1v[TPW];
#pragma unroll
    for (int u = 0; u < TPW; ++u) {
        const int t = wv * TPW + u;
        const int nl = t / ptiles;
        pv[u] = ((t - nl * ptiles) << 5) + 2 * col;
        nlv[u] = t < ntp ? nl : -1;   // pv < P: P >= 64 here; wave-uniform
        const float2 w01 = nlv[u] >= 0 ? *reinterpret_cast<const float2*>(k.win + pv[u]) : make_float2(0.f, 0.f);
        w0v[u] = w01.x;
        w1v[u] = w01.y;
    }
    const size_t NPc = (size_t)g.cpitch;
    // per-lane byte offsets of this lane's (channel, pulse pair) inside a cube: loop-invariant,
    // so a tile's load issue is scalar sample offsets + buffer loads and writes no VGPR but xv
    // (a VGPR temporary there could be a pending z store's data register: WAR = vmcnt wait)
    unsigned loff[TPW][NJ];
#pragma unroll
    for (int u = 0; u < TPW; ++u)
#pragma unroll
        for (int j = 0; j < NJ; ++j) loff[u][j] = (unsigned)(((size_t)min(4 * j + grp, C - 1) * NPc + pv[u]) * 8u);
    const unsigned cube_bytes = (unsigned)((size_t)C * NPc * 8u);
    float4 xv[TPW][NJ];
    bool vld[TPW];   // wave-uniform: sub-tile u of the tile in flight lies inside the used samples
    auto issue = [&](int TT) {   // cube loads of tile TT (fsf:93 operands) into xv
        const int f = __builtin_amdgcn_readfirstlane(TT / g.ntiles), tile = TT - f * g.ntiles;
        const __amdgpu_buffer_rsrc_t xr = buf_rsrc(fp.in[f], cube_bytes);
#pragma unroll
        for (int u = 0; u < TPW; ++u) {
            const int np = tile * NT + nlv[u];
            vld[u] = nlv[u] >= 0 && np < g.nU;
            if (vld[u]) {   // no else: zeroing xv here would wait (vmcnt) on the pending z stores
                const int soff = used_sample(g, np) * P * 8;
#pragma unroll
                for (int j = 0; j < NJ; ++j) {   // non-temporal: the cube is read exactly once
                    const u32x4 t = __builtin_amdgcn_raw_buffer_load_b128(xr, (int)loff[u][j], soff, 2);
                    xv[u][j] = make_float4(__uint_as_float(t.x), __uint_as_float(t.y), __uint_as_float(t.z),
                                           __uint_as_float(t.w));
                }
            }
        }
    };
    auto dbf = [&](float2* buf) {   // MFMA DBF + window of xv into buf (padded rows, K1_SH)
        float* Yf = reinterpret_cast<float*>(buf);
#pragma unroll
        for (int u = 0; u < TPW; ++u) {
            if (nlv[u] < 0) continue;
            if (!vld[u]) {   // samples past the used ones: zero columns, like k1_dbf_mtd's n = -1
                const int p = pv[u];
                const int i0 = p + (p >> K1_SH), i1 = (p + 1) + ((p + 1) >> K1_SH);
#pragma unroll
                for (int mb = 0; mb < MB; ++mb)
#pragma unroll
                    for (int i = 0; i < 4; ++i) {
                        const int m = 4 * grp + i, b = mb * 8 + (m & 7);
                        if (b < B) {
                            float* colp = Yf + 2 * (b * NT + nlv[u]) * Ppad + (m >> 3);
                            colp[2 * i0] = 0.f;
                            colp[2 * i1] = 0.f;
                        }
                    }
                continue;
            }
            f32x4 acc[MB][2];
#pragma unroll
            for (int mb = 0; mb < MB; ++mb) {
                acc[mb][0] = f32x4{0.f, 0.f, 0.f, 0.f};
                acc[mb][1] = acc[mb][0];
#pragma unroll
                for (int j = 0; j < NJ; ++j) {
                    acc[mb][0] = __builtin_amdgcn_mfma_f32_16x16x4f32(are[mb][j], xv[u][j].x, acc[mb][0], 0, 0, 0);
                    acc[mb][0] = __builtin_amdgcn_mfma_f32_16x16x4f32(aim[mb][j], xv[u][j].y, acc[mb][0], 0, 0, 0);
                    acc[mb][1] = __builtin_amdgcn_mfma_f32_16x16x4f32(are[mb][j], xv[u][j].z, acc[mb][1], 0, 0, 0);
                    acc[mb][1] = __builtin_amdgcn_mfma_f32_16x16x4f32(aim[mb][j], xv[u][j].w, acc[mb][1], 0, 0, 0);
                }
            }
            const int p = pv[u];
            const int i0 = p + (p >> K1_SH), i1 = (p + 1) + ((p + 1) >> K1_SH);
#pragma unroll
            for (int mb = 0; mb < MB; ++mb)
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const int m = 4 * grp + i;
                    const int b = mb * 8 + (m & 7);
                    if (b < B) {
                        float* colp = Yf + 2 * (b * NT + nlv[u]) * Ppad + (m >> 3);
                        colp[2 * i0] = acc[mb][0][i] * w0v[u];
                        colp[2 * i1] = acc[mb][1][i] * w1v[u];
                    }
                }
        }
    };
    const int zslab = P * NT, lgNT = ilog2(NT), half = P >> 1;
    // diagnostic (RSP_TRACE_FILE): stamp 0 = start, 1 / 2 = summed FFT+store / DBF phase ticks
    // (not timestamps), 3 = end; thread 0, after the barriers that close each phase
    const bool tr = fp.trace != nullptr && threadIdx.x == 0;
    unsigned long long t0 = tr ? __builtin_amdgcn_s_memrealtime() : 0, tfft = 0, tdbf = 0, tiss = 0;
    issue(T);
    dbf(Y);
    __syncthreads();
    const unsigned long long tpro = tr ? __builtin_amdgcn_s_memrealtime() : 0;
    int cur = 0;
    for (; T < total; T += gridDim.x) {
        const int Tn = T + gridDim.x;
        const unsigned long long ti = tr ? __builtin_amdgcn_s_memrealtime() : 0;
        if (Tn < total) issue(Tn);   // next tile's loads fly during this tile's FFT + z stores
        if (tr) tiss += __builtin_amdgcn_s_memrealtime() - ti;
        const int f = __builtin_amdgcn_readfirstlane(T / g.ntiles), tile = T - f * g.ntiles;
        if (tile == 0 && threadIdx.x == 0 && fp.count[f]) *fp.count[f] = 0;   // K3's detection counter
        float2* __restrict__ z = fp.z[f];
        const StoreZ sz{buf_rsrc(z, (unsigned)B * g.ntiles * zslab * 8u), lgNT, g.ntiles, tile, P, half};
        const unsigned long long ta = tr ? __builtin_amdgcn_s_memrealtime() : 0;
        fft_passes<LGP, 0, 0, 16, false, K1_SH, K1_THREADS>(Y + cur * bufsz, Ppad, B * NT, twl,
                                                           StoreLds{Y + cur * bufsz}, sz);   // ends with a barrier
        const unsigned long long tb = tr ? __builtin_amdgcn_s_memrealtime() : 0;
        if (Tn < total) dbf(Y + (nbuf == 2 ? (cur ^ 1) : 0) * bufsz);
        __syncthreads();
        if (tr) {
            tfft += tb - ta;
            tdbf += __builtin_amdgcn_s_memrealtime() - tb;
        }
        if (nbuf == 2) cur ^= 1;
    }
    if (tr) {
        unsigned long long* o = fp.trace + (size_t)blockIdx.x * 4;
        o[0] = t0;
        o[1] = (g.dbg & 16384) ? tpro - t0 : (g.dbg & 32768) ? tiss : tfft;   // 16384 / 32768: prologue / issue ticks
        o[2] = tdbf;
        o[3] = __builtin_amdgcn_s_memrealtime();
    }
}

// ======================================================================================
// K2: pulse compression of every row (fsf:101-126)
// ======================================================================================
__device__ __forceinline__ float cabsf(float2 a) { return sqrtf(a.x * a.x + a.y * a.y); }

struct StoreRdm {   // last inverse pass: keep outputs i in [Lh-1, Lh-1+V) that map to gates < gend;
                    // also writes |x| (the CFAR input, fsf:184-185) into the magnitude map.
                    // Branch-free: rejected outputs get an out-of-range buffer offset.
    __amdgpu_buffer_rsrc_t rdm, mag; int G; int Gp; int row0; int rows_total; int Lh1; int g0; int gend;
    __device__ __forceinline__ void put(int, int row, int o, int, f2 x) const {
        const int gg = g0 + o - Lh1;
        const int rho = row0 + row;
        const bool ok = o >= Lh1 && gg < gend && rho < rows_total;
        buf_st_f2<RSP_ST_AUX>(rdm, ok ? (unsigned)(rho * G + gg) * 8u : RSP_OOB, x);
        buf_st_f1(mag, ok ? (unsigned)(rho * Gp + gg) * 4u : RSP_OOB, fast_abs(x));
    }
};

#ifndef K2_SH
#define K2_SH 5   // one pad complex per 32 (tools/lds_conflicts.py)
#endif
#define K2_LDS_DATA (RSP_K2_POINTS + (RSP_K2_POINTS >> K2_SH))
#define K2_LDS_TW 4096       // >= tw_total(log2 M) + tw_total(log2 M, reversed) for M <= 2048
#define K2_LDS_TW_CMP 1408   // the same for compact tables
#define K2_MAXM 2048

// ---- mixed-radix overlap-save blocks (M = 5 * 2^k): three Stockham passes of radices
// (RA, RB, RC) forward and (RC, RB, RA) inverse, RC = 10.  Butterfly counts M / R and partial
// products Ns need not be powers of two, so every LDS index is padded per element.
#define K2M_POINTS K2M_POINTS_HOST   // complex points per mixed-radix workgroup (10 per thread)

template <int R, bool INV, int NB, int M, int NS, int NTHR>
__device__ __forceinline__ void shm_load(const float2* buf, int rs, int nrows, const float2* tw, f2 (&v)[NB][R]) {
    constexpr int nb = M / R;
    const int total = nb * nrows;
#pragma unroll
    for (int t = 0; t < NB; ++t) {
        const int beta = threadIdx.x + t * NTHR;
        if (beta < total) {
            const int row = beta / nb, j = beta - row * nb;
            const float2* rowp = buf + row * rs;
            f2 w[R];
            if (NS > 1) load_tw<R, INV, true>(tw + (j % NS) * tw_row(R, true), w);
#pragma unroll
            for (int r = 0; r < R; ++r) {
                f2 x = tof2(rowp[lidx<K2_SH>(j + r * nb)]);
                if (r > 0 && NS > 1) x = vmul(x, w[r]);
                v[t][r] = x;
            }
        }
    }
}

template <int R, bool INV, int NB, int M, int NS, int NTHR, class St>
__device__ __forceinline__ void shm_store(f2 (&v)[NB][R], int rs, int nrows, const St& st) {
    constexpr int nb = M / R;
    const int total = nb * nrows;
#pragma unroll
    for (int t = 0; t < NB; ++t) {
        const int beta = threadIdx.x + t * NTHR;
        if (beta < total) {
            const int row = beta / nb, j = beta - row * nb;
            Dft<R, INV>::run(v[t]);
            const int idxD = (j / NS) * (NS * R) + j % NS;
#pragma unroll
            for (int r = 0; r < R; ++r) {
                const int o = idxD + r * NS;
                st.put(t * R + r, row, o, row * rs + lidx<K2_SH>(o), v[t][r]);
            }
        }
    }
}

template <int R, bool INV, int NB, int M, int NS, int NTHR, class St>
__device__ __forceinline__ void shm_pass(float2* buf, int rs, int nrows, const float2* tw, const St& st) {
    f2 v[NB][R];
    shm_load<R, INV, NB, M, NS, NTHR>(buf, rs, nrows, tw, v);
    __syncthreads();
    shm_store<R, INV, NB, M, NS, NTHR>(v, rs, nrows, st);
    __syncthreads();
}

// Twiddle table sizes / offsets of the mixed plans (must match build_mixed_twiddles() in
// rsp_plan.cpp): forward tables, then inverse; pass q >= 1 owns Ns_q rows of tw_row(R_q).
constexpr int twm_fwd(int RA, int RB, int RC) { return RA * tw_row(RB, true) + RA * RB * tw_row(RC, true); }

template <int M, int RA, int RB, int RC, int NTHR, int PTSW>
__device__ __forceinline__ void k2m_fft_job(const Geometry& g, const DevConsts& k, const SegDesc& sd, const K2Job& job,
                                            const float2* __restrict__ z, float2* __restrict__ rdm,
                                            float* __restrict__ mag, int row0, int rows_total, float2* L,
                                            const FramePtrs& fp) {
    static_assert(RA * RB * RC == M, "mixed plan must factor M");
    constexpr int rows = PTSW / M;
    constexpr int PTS = PTSW / NTHR;
    constexpr int rs = M + (M >> K2_SH);
    constexpr int NBA = (PTS + RA - 1) / RA, NBB = (PTS + RB - 1) / RB, NBC = (PTS + RC - 1) / RC;
    constexpr int nb0 = M / RA;
    const int P = g.P, G = g.G;
    const int lo = sd.lo, hi = sd.hi, off = sd.off;
    const int tid = threadIdx.x;
    const int Lh1 = sd.Lh - 1;
    const int g0 = sd.ga + job.blk * sd.V;
    const int a = sd.seg_lo + g0 - Lh1;   // sample index of u[0]
    const float2* twf = k.twM + sd.tw_off;
    const float2* twi = twf + twm_fwd(RA, RB, RC);
    const __amdgpu_buffer_rsrc_t zr = buf_rsrc(z, (unsigned)g.B * g.ntiles * P * g.NT * 8u);
    // forward pass 0 (Ns = 1) straight from z
    f2 v0[NBA][RA];
#pragma unroll
    for (int t = 0; t < NBA; ++t) {
        const int beta = tid + t * NTHR;
        const int rl = beta / nb0, j = beta - rl * nb0;
        const int rho = row0 + rl;
        const int b = rho / P, v = rho - b * P;
        const bool live = beta < rows * nb0 && rho < rows_total;
#pragma unroll
        for (int r = 0; r < RA; ++r) {
            const int n = a + j + r * nb0;
            const bool ok = live && n >= lo && n <= hi;
            v0[t][r] = buf_ld_f2(zr, ok ? (unsigned)zaddr(g, b, v, n - lo + off) * 8u : RSP_OOB);
        }
    }
    // H for the last forward pass's outputs j + r M / RC (1/M folded in)
    f2 hreg[NBC][RC];
#pragma unroll
    for (int t = 0; t < NBC; ++t) {
        const int j = (tid + t * NTHR) % (M / RC);
#pragma unroll
        for (int r = 0; r < RC; ++r) hreg[t][r] = tof2(k.H[sd.H_off + j + r * (M / RC)]);
    }
    shm_store<RA, false, NBA, M, 1, NTHR>(v0, rs, rows, StoreLds{L});
    __syncthreads();
    trace_stamp(fp, 1);
    shm_pass<RB, false, NBB, M, RA, NTHR>(L, rs, rows, twf, StoreLds{L});
    {   // fused: forward last pass, x H, inverse pass 0 (same butterflies)
        f2 v[NBC][RC];
        shm_load<RC, false, NBC, M, RA * RB, NTHR>(L, rs, rows, twf + RA * tw_row(RB, true), v);
        __syncthreads();
#pragma unroll
        for (int t = 0; t < NBC; ++t) {
            Dft<RC, false>::run(v[t]);
#pragma unroll
            for (int r = 0; r < RC; ++r) v[t][r] = vmul(v[t][r], hreg[t][r]);
        }
        shm_store<RC, true, NBC, M, 1, NTHR>(v, rs, rows, StoreLds{L});
        __syncthreads();
    }
    trace_stamp(fp, 2);
    shm_pass<RB, true, NBB, M, RC, NTHR>(L, rs, rows, twi, StoreLds{L});
    const int gend = min(sd.gb, g0 + sd.V);
    shm_pass<RA, true, NBA, M, RC * RB, NTHR>(
        L, rs, rows, twi + RC * tw_row(RB, true),
        StoreRdm{buf_rsrc(rdm, (unsigned)rows_total * G * 8u), buf_rsrc(mag, (unsigned)rows_total * g.Gp * 4u), G, g.Gp,
                 row0, rows_total, Lh1, g0, gend});
    trace_stamp(fp, 3);
}

// Mixed-radix jobs as a launch of their own (jobs [g.mix_job0, njobs), workgroups from
// g.nwg_k2_pow2): 2 rows x 2560 points over 320 threads, so every radix-16 pass keeps all
// threads busy (16 points each) and the radix-10 passes 80 % of them.
#ifndef K2M_THREADS
#define K2M_THREADS 320
#endif
template <int M, int RA, int RB, int RC>
__global__ __launch_bounds__(K2M_THREADS, K2M_THREADS > 320 ? 2 : 3) void k2m_pc(Geometry g, DevConsts k, FramePtrs fp, int rows_total) {
    extern __shared__ __attribute__((aligned(16))) float2 L[];
    const int f = blockIdx.y;
    const int wg = g.nwg_k2_pow2 + blockIdx.x;
    int ji = g.mix_job0;
    while (ji + 1 < g.njobs && wg >= g.jobs[ji + 1].wg_begin) ++ji;
    const K2Job job = g.jobs[ji];
    const SegDesc& sd = g.segs[job.seg];
    const int row0 = (wg - job.wg_begin) * sd.rows_per_wg;
    trace_stamp(fp, 0);
    k2m_fft_job<M, RA, RB, RC, K2M_THREADS, 2 * M>(g, k, sd, job, fp.z[f], fp.rdm[f], fp.mag[f], row0, rows_total, L, fp);
}

// One overlap-save block of one FFT segment for RSP_K2_POINTS / 2^LGM adjacent rows.
// LDS round trips: forward pass 0 runs on the samples as loaded from z; the forward FFT's
// last pass, the filter-spectrum product and the inverse FFT's first pass (radices in
// reverse order, so that pass has the same butterflies) run in registers back to back;
// the inverse FFT's last pass stores the kept gates to HBM.  2 (log2 M / 4) round trips
// instead of 2 (log2 M / 4) + 3.
template <int LGM, bool TWG, bool CMP>
__device__ __forceinline__ void k2_fft_job(const Geometry& g, const DevConsts& k, const SegDesc& sd, const K2Job& job,
                                           const float2* __restrict__ z, float2* __restrict__ rdm,
                                           float* __restrict__ mag, int row0, int rows_total, float2* L,
                                           const FramePtrs& fp) {
    constexpr int M = 1 << LGM;
    constexpr int rows = RSP_K2_POINTS / M;
    constexpr int rs = M + (M >> K2_SH);
    constexpr int NP = n_passes(LGM);
    static_assert(NP >= 2, "overlap-save block needs >= 2 FFT passes");
    constexpr int RB0 = rad_bits(LGM, 0), R0 = 1 << RB0, NB0 = 16 / R0, nb0 = M / R0;
    constexpr int RBL = rad_bits(LGM, NP - 1), RL = 1 << RBL, NBL = 16 / RL;   // last forward pass
    const int P = g.P, G = g.G;
    const int lo = sd.lo, hi = sd.hi, off = sd.off;
    const int tid = threadIdx.x;
    const int Lh1 = sd.Lh - 1;
    const int g0 = sd.ga + job.blk * sd.V;
    const int a = sd.seg_lo + g0 - Lh1;           // sample index of u[0]
    // twiddle tables: LDS copy, or (TWG) read in place from global memory (L1/L2 resident)
    float2* twl = TWG ? const_cast<float2*>(k.twM + sd.tw_off) : L + K2_LDS_DATA;
    // every global load of the workgroup in flight together: the 16 samples of this thread's
    // pass-0 butterflies, its 16 filter-spectrum values (for the fused middle pass) and the
    // twiddle tables
    f2 v0[NB0][R0];
    const int lgNT = ilog2(g.NT);
    const __amdgpu_buffer_rsrc_t zr = buf_rsrc(z, (unsigned)g.B * g.ntiles * P * g.NT * 8u);
#pragma unroll
    for (int t = 0; t < NB0; ++t) {
        const int beta = tid + t * K2_THREADS;
        const int rl = beta / nb0, j = beta & (nb0 - 1);
        const int rho = row0 + rl;
        const int b = rho / P, v = rho - b * P;
        // z index of sample n0 + r nb0: when NT | nb0 the tile advances by nb0/NT per r and the
        // in-tile slot is fixed, so element r sits at zb + r (nb0 P) (one multiply per thread)
        const int np0 = a + j - lo + off;
        const int zb = ((b * g.ntiles + (np0 >> lgNT)) * P + v) * g.NT + (np0 & (g.NT - 1));
        // branch-free: every lane loads (a valid address when masked) and selects
        if ((nb0 & (g.NT - 1)) == 0) {   // uniform
#pragma unroll
            for (int r = 0; r < R0; ++r) {
                const int n = a + j + r * nb0;
                const bool ok = rho < rows_total && n >= lo && n <= hi;
                v0[t][r] = buf_ld_f2(zr, ok ? (unsigned)(zb + r * nb0 * P) * 8u : RSP_OOB);
            }
        } else {
#pragma unroll
            for (int r = 0; r < R0; ++r) {
                const int n = a + j + r * nb0;
                const bool ok = rho < rows_total && n >= lo && n <= hi;
                v0[t][r] = buf_ld_f2(zr, ok ? (unsigned)zaddr(g, b, v, n - lo + off) * 8u : RSP_OOB);
            }
        }
    }
    // H for the last forward pass's outputs j + r M/RL; butterflies t and t + (M/RL)/NTHR of a
    // thread have the same j (different rows), so only the distinct ones are loaded
    constexpr int NHT = (M / RL) / K2_THREADS >= NBL ? NBL : ((M / RL) / K2_THREADS > 0 ? (M / RL) / K2_THREADS : 1);
    f2 hreg[NHT * RL];
#pragma unroll
    for (int t = 0; t < NHT; ++t) {
        const int j = (tid + t * K2_THREADS) & (M / RL - 1);   // last pass: Ns = nb = M / RL, idxD = j
#pragma unroll
        for (int r = 0; r < RL; ++r) hreg[t * RL + r] = tof2(k.H[sd.H_off + j + r * (M / RL)]);
    }
    constexpr int NTWF = tw_total(LGM, false, CMP);
    constexpr int NTW = NTWF + tw_total(LGM, true, CMP);
    static_assert(NTW <= (CMP ? K2_LDS_TW_CMP : K2_LDS_TW), "K2 twiddle tables exceed their LDS slot");
    constexpr int NT_TAB = TWG ? 0 : (NTW + K2_THREADS - 1) / K2_THREADS;
    float2 tv[NT_TAB > 0 ? NT_TAB : 1];
#pragma unroll
    for (int u = 0; u < NT_TAB; ++u) {
        const int i = tid + u * K2_THREADS;
        if (i < NTW) tv[u] = k.twM[sd.tw_off + i];
    }
    // forward pass 0 (Ns = 1, no twiddles) straight from the loaded samples
    sh_store<R0, false, NB0, K2_SH, K2_THREADS, LGM, 0>(v0, rs, rows, StoreLds{L});
#pragma unroll
    for (int u = 0; u < NT_TAB; ++u) {
        const int i = tid + u * K2_THREADS;
        if (i < NTW) twl[i] = tv[u];
    }
    __syncthreads();
    trace_stamp(fp, 1);
    // forward passes 1 .. NP-2
    fft_range<LGM, 1, NP - 1, RB0, 16, false, false, K2_SH, K2_THREADS, CMP>(L, rs, rows, twl, StoreLds{L},
                                                                               StoreLds{L});
    // fused: forward last pass, x H (1/M folded in), inverse pass 0 of the reversed plan
    {
        f2 v[NBL][RL];
        sh_load<RL, false, NBL, K2_SH, K2_THREADS, LGM, LGM - RBL, CMP>(L, rs, rows,
                                                                       twl + tw_pass_off(LGM, NP - 1, false, CMP), v);
        __syncthreads();
#pragma unroll
        for (int t = 0; t < NBL; ++t) {
            Dft<RL, false>::run(v[t]);
#pragma unroll
            for (int r = 0; r < RL; ++r) v[t][r] = vmul(v[t][r], hreg[(t % NHT) * RL + r]);
        }
        sh_store<RL, true, NBL, K2_SH, K2_THREADS, LGM, 0>(v, rs, rows, StoreLds{L});
        __syncthreads();
    }
    trace_stamp(fp, 2);
    // inverse passes 1 .. NP-1 (reversed radices); the last keeps the valid overlap-save
    // outputs = stitched gates
    const int gend = min(sd.gb, g0 + sd.V);
    fft_range<LGM, 1, NP, RBL, 16, true, true, K2_SH, K2_THREADS, CMP>(
        L, rs, rows, twl + NTWF, StoreLds{L}, StoreRdm{buf_rsrc(rdm, (unsigned)rows_total * G * 8u),
                                                      buf_rsrc(mag, (unsigned)rows_total * g.Gp * 4u), G, g.Gp,
                                                      row0, rows_total, Lh1, g0, gend});
    trace_stamp(fp, 3);
}

template <bool TWG, bool CMP>
__global__ __launch_bounds__(K2_THREADS, 512 / K2_THREADS) void k2_pc(Geometry g, DevConsts k, FramePtrs fp, int rows_total) {
    extern __shared__ __attribute__((aligned(16))) float2 L[];   // data | twiddles (M) | H (M)
    const int f = blockIdx.y;
    const int wg = blockIdx.x;
    int ji = 0;
    while (ji + 1 < g.njobs && wg >= g.jobs[ji + 1].wg_begin) ++ji;
    const K2Job job = g.jobs[ji];
    const SegDesc& sd = g.segs[job.seg];
    const int rows = sd.rows_per_wg;
    const int row0 = (wg - job.wg_begin) * rows;
    trace_stamp(fp, 0);
    const float2* __restrict__ z = fp.z[f];
    float2* __restrict__ rdm = fp.rdm[f];
    float* __restrict__ mag = fp.mag[f];
    const int P = g.P, G = g.G;
    const int lo = sd.lo, hi = sd.hi, off = sd.off;
    const int tid = threadIdx.x;

    if (sd.type == 1 && sd.mixM) {
        switch (sd.mixM) {
            case 640: k2m_fft_job<640, 8, 8, 10, K2_THREADS, K2M_POINTS>(g, k, sd, job, z, rdm, mag, row0, rows_total, L, fp); break;
            case 1280: k2m_fft_job<1280, 16, 8, 10, K2_THREADS, K2M_POINTS>(g, k, sd, job, z, rdm, mag, row0, rows_total, L, fp); break;
            default: k2m_fft_job<2560, 16, 16, 10, K2_THREADS, K2M_POINTS>(g, k, sd, job, z, rdm, mag, row0, rows_total, L, fp); break;
        }
    } else if (sd.type == 1) {
#ifdef K2_ONLY_LGM   // ISA inspection builds: one block size only
        k2_fft_job<K2_ONLY_LGM, TWG, CMP>(g, k, sd, job, z, rdm, mag, row0, rows_total, L, fp);
        if (sd.logM >= 0) return;
#endif
        switch (sd.logM) {
            case 6: k2_fft_job<6, TWG, CMP>(g, k, sd, job, z, rdm, mag, row0, rows_total, L, fp); break;
            case 7: k2_fft_job<7, TWG, CMP>(g, k, sd, job, z, rdm, mag, row0, rows_total, L, fp); break;
            case 8: k2_fft_job<8, TWG, CMP>(g, k, sd, job, z, rdm, mag, row0, rows_total, L, fp); break;
            case 9: k2_fft_job<9, TWG, CMP>(g, k, sd, job, z, rdm, mag, row0, rows_total, L, fp); break;
            case 10: k2_fft_job<10, TWG, CMP>(g, k, sd, job, z, rdm, mag, row0, rows_total, L, fp); break;
            default: k2_fft_job<11, TWG, CMP>(g, k, sd, job, z, rdm, mag, row0, rows_total, L, fp); break;
        }
    } else {
        // direct FIR (narrow segment): filter() + circshift(-fir_delay) (fsf:111-112).  Each
        // staged row carries ntaps - 1 leading zeros (filter()'s zero state / samples before lo),
        // so the tap loop is branch-free.
        const int W = hi - lo + 1;
        const int PADL = sd.ntaps - 1, WP = W + PADL;
        const int nw = rows * WP;
        for (int e0 = 0; e0 < nw; e0 += 16 * K2_THREADS) {
            float2 val[16];
#pragma unroll
            for (int u = 0; u < 16; ++u) {
                const int e = e0 + tid + u * K2_THREADS;
                val[u] = make_float2(0.f, 0.f);
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
        float* tp = reinterpret_cast<float*>(L + nw);   // taps: LDS broadcast reads
        for (int e = tid; e < sd.ntaps; e += K2_THREADS) tp[e] = k.taps[sd.taps_off + e];
        __syncthreads();
        trace_stamp(fp, 1);
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
            const float2* row = L + rl * WP + PADL - lo + sd.seg_lo;   // row[kk] = x(seg_lo + kk)
            if (q0 + 4 <= nout && kk0 + 3 < sd.Ls) {
                const float2* xr = row + kk0;
                f2 w0 = tof2(xr[0]), w1 = tof2(xr[1]), w2 = tof2(xr[2]), w3 = tof2(xr[3]);
                float t = tp[0];
                f2 a0 = t * w0, a1 = t * w1, a2 = t * w2, a3 = t * w3;
#pragma unroll 4
                for (int j = 1; j < sd.ntaps; ++j) {
                    w3 = w2; w2 = w1; w1 = w0;
                    w0 = tof2(xr[-j]);
                    t = tp[j];
                    a0 += t * w0; a1 += t * w1; a2 += t * w2; a3 += t * w3;
                }
                float2* ro = rdm + (size_t)rho * G + gg0;
                float* mo = mag + (size_t)rho * g.Gp + gg0;
                ro[0] = fromf2(a0); ro[1] = fromf2(a1); ro[2] = fromf2(a2); ro[3] = fromf2(a3);
                mo[0] = fast_abs(a0); mo[1] = fast_abs(a1); mo[2] = fast_abs(a2); mo[3] = fast_abs(a3);
            } else {
                for (int q = 0; q < 4 && q0 + q < nout; ++q) {
                    const int gg = gg0 + q;
                    int kk = (gg + sd.delay) % sd.Ls;
                    if (kk < 0) kk += sd.Ls;
                    const float2* xr = row + kk;
                    f2 acc = f2{0.f, 0.f};
                    for (int j = 0; j < sd.ntaps; ++j) acc += tp[j] * tof2(xr[-j]);
                    rdm[(size_t)rho * G + gg] = fromf2(acc);
                    mag[(size_t)rho * g.Gp + gg] = fast_abs(acc);
                }
            }
        }
        trace_stamp(fp, 2);
        trace_stamp(fp, 3);
    }
}

// ======================================================================================
// K3: GOCA-CFAR on adjacent-beam sums + compaction + S9 estimation
// ======================================================================================
// Peak of MATLAB interp1(...,'spline') (not-a-knot) sampled at step 1/interp over n
// equally spaced points (fsf:257-260, 272-275); returns the first-argmax abscissa.
template <int INTERP>
__device__ double spline_peak(const double* y, int n) {
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
        const double d1 = y[1] - y[0], d2 = y[2] - 2.0 * y[1] + y[0];
        const double d3 = (n == 4) ? y[3] - 3.0 * y[2] + 3.0 * y[1] - y[0] : 0.0;
        // Newton form about x = 0 expanded at each integer knot i
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const double x = i;
            c0[i] = y[0] + x * d1 + x * (x - 1.0) * 0.5 * d2 + x * (x - 1.0) * (x - 2.0) * (1.0 / 6.0) * d3;
            c1[i] = d1 + (2.0 * x - 1.0) * 0.5 * d2 + (3.0 * x * x - 6.0 * x + 2.0) * (1.0 / 6.0) * d3;
            c2[i] = 0.5 * d2 + (3.0 * x - 3.0) * (1.0 / 6.0) * d3;
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

// S9 of one detection from the workgroup's S tile (fsf:237-290).
__device__ __forceinline__ void s9_estimate(const DevConsts& k, const float* S, int W, int c0, int P, int G, int Gp,
                                            int v, int r, int pair, const float* __restrict__ MA,
                                            const float* __restrict__ MB, DevDet* out) {
    const int c = r - c0;
    // the 5-cell windows clipped to the map (fsf:241-250): cells first .. first + n - 1
    const int rfirst = max(r - 2, 0), nrc = min(r + 2, G - 1) - rfirst + 1;
    const int vfirst = max(v - 2, 0), nvc = min(v + 2, P - 1) - vfirst + 1;
    double yr[5], yv[5];
#pragma unroll
    for (int j = 0; j < 5; ++j) {
        yr[j] = j < nrc ? (double)S[v * W + (rfirst - c0) + j] : 0.0;
        yv[j] = j < nvc ? (double)S[(vfirst + j) * W + c] : 0.0;
    }
    const double rmax = (nrc < 3) ? (double)r : rfirst + spline_peak<8>(yr, nrc);
    const double vmax = (nvc < 3) ? (double)v : vfirst + spline_peak<4>(yv, nvc);
    // amplitude monopulse on the integer cell (fsf:282-290)
    const double SA = (double)MA[(size_t)v * Gp + r];
    const double SB = (double)MB[(size_t)v * Gp + r];
    const double ratio = (SA - SB) / (SA + SB + 2.220446049250313e-16);
    DevDet d;
    d.v_idx = v + 1;
    d.r_idx = r + 1;
    d.pair_idx = pair + 1;
    d.reserved = 0;
    d.amp = (double)S[v * W + c];
    d.range = k.range_axis[r] + (rmax - r) * k.deltaR;
    d.velocity = k.velocity_axis[v] + (vmax - v) * k.deltaV;
    d.angle = 0.5 * (k.beam_angles[pair] + k.beam_angles[pair + 1]) + k.klut[pair] * ratio;
    *out = d;
}

// Out-of-line copy for the queue-overflow path (pathological detection densities), so the
// CFAR loops do not carry an inlined S9 body.
__device__ __attribute__((noinline)) void s9_estimate_ool(const DevConsts& k, const float* S, int W, int c0, int P,
                                                          int G, int Gp, int v, int r, int pair, const float* MA,
                                                          const float* MB, DevDet* out) {
    s9_estimate(k, S, W, c0, P, G, Gp, v, r, pair, MA, MB, out);
}

#define K3_QCAP 1024
#define K3_VEC 12   // float4 loads per beam per thread in flight

constexpr int floor4(int x) { return x >= 0 ? (x & ~3) : -((-x + 3) & ~3); }

// RR/RV/GR/GV = reference/guard cell counts when known at compile time (the reference's
// 5/5/10/10, v8:45-46), 0 = runtime.  Tiles: RT range cells x all P Doppler cells of one beam
// pair, tile starts aligned to 4 cells so that the magnitude rows load as float4.
template <int RR, int RV, int GR, int GV>
__global__ __launch_bounds__(RSP_THREADS, 3) void k3_cfar(Geometry g, DevConsts k, FramePtrs fp) {
    extern __shared__ __attribute__((aligned(16))) float S[];   // [P][W] | queue[K3_QCAP] | qn, base
    constexpr bool FAST = RR > 0 && RV > 0 && GR > 0 && GV > 0;
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
    const int tile = col % ntile, f = col / ntile;
    const int P = g.P, G = g.G, W = g.cfar_W, hR = g.cfar_hR, RT = g.cfar_RT;
    const int rR = RR ? RR : g.refR, gR = GR ? GR : g.guardR, rV = RV ? RV : g.refV, gV = GV ? GV : g.guardV;
    const int rc0 = rR + gR;                           // first cell under test (0-based)
    const int tstart = (rc0 & ~3) + tile * RT;         // multiple of 4
    const int c0 = tstart - hR;                        // tile column 0 (multiple of 4; may be < 0)
    const int cut_lo = max(tstart, rc0), cut_hi = min(tstart + RT, G - rc0);
    int* queue = reinterpret_cast<int*>(S + P * W);
    int* qn = queue + K3_QCAP;
    const int Gp = g.Gp;
    const float* __restrict__ MA = fp.mag[f] + (size_t)pair * P * Gp;   // |RDM| of beams pair, pair+1
    const float* __restrict__ MB = MA + (size_t)P * Gp;
    trace_stamp(fp, 0);
    if (threadIdx.x == 0) qn[0] = 0;
    // ---- load S = |A| + |B| (fsf:184-187) from the magnitude maps: 16 B per lane,
    //      K3_VEC float4 of each beam in flight per thread
    {
        const int W4 = W >> 2, n4 = P * W4;
        for (int e0 = 0; e0 < n4; e0 += K3_VEC * RSP_THREADS) {
            float4 xa[K3_VEC], xb[K3_VEC];
#pragma unroll
            for (int u = 0; u < K3_VEC; ++u) {
                const int e = e0 + threadIdx.x + u * RSP_THREADS;
                xa[u] = make_float4(0.f, 0.f, 0.f, 0.f);
                xb[u] = xa[u];
                if (e < n4) {
                    const int v = e / W4, r = c0 + 4 * (e - v * W4);
                    if (r >= 0 && r < G) {   // rows are padded to Gp (multiple of 4): r + 3 < Gp
                        xa[u] = *reinterpret_cast<const float4*>(MA + (size_t)v * Gp + r);
                        xb[u] = *reinterpret_cast<const float4*>(MB + (size_t)v * Gp + r);
                        if (r + 1 >= G) { xa[u].y = 0.f; xb[u].y = 0.f; }
                        if (r + 2 >= G) { xa[u].z = 0.f; xb[u].z = 0.f; }
                        if (r + 3 >= G) { xa[u].w = 0.f; xb[u].w = 0.f; }
                    }
                }
            }
#pragma unroll
            for (int u = 0; u < K3_VEC; ++u) {
                const int e = e0 + threadIdx.x + u * RSP_THREADS;
                if (e < n4)
                    reinterpret_cast<float4*>(S)[e] =
                        make_float4(xa[u].x + xb[u].x, xa[u].y + xb[u].y, xa[u].z + xb[u].z, xa[u].w + xb[u].w);
            }
        }
    }
    __syncthreads();
    trace_stamp(fp, 1);
    const int v0 = rV + gV, v1 = P - rV - gV;
    if (v1 <= v0 || cut_hi <= cut_lo) return;
    const float fR = (float)rR, fV = (float)rV;
    // mean() = sum / n over the slices of fsf:197-203 (max(a/n, b/n) = max(a, b)/n); the
    // division is a multiply by 1/n (<= 1 ulp from the quotient: only cells within that of the
    // threshold can decide differently, the fp32-vs-fp64 band the parity tests allow)
    const float iR = 1.0f / fR, iV = 1.0f / fV;
#define K3_HIT(V, C, CUT, LR, TR, LV, TV)                                                               \
    do {                                                                                                \
        const float nR_ = fmaxf(LR, TR) * iR, nV_ = fmaxf(LV, TV) * iV;                                 \
        if ((CUT) > g.T * fmaxf(nR_, nV_)) {                                                            \
            const int qi = atomicAdd(qn, 1);                                                            \
            if (qi < K3_QCAP) {                                                                         \
                queue[qi] = ((V) << 16) | (C);                                                          \
            } else { /* queue overflow (pathological): estimate in place */                             \
                const int idx = atomicAdd(fp.count[f], 1);                                              \
                if (idx < g.max_dets)                                                                   \
                    s9_estimate_ool(k, S, W, c0, P, G, Gp, V, c0 + (C), pair, MA, MB, &fp.dets[f][idx]); \
            }                                                                                           \
        }                                                                                               \
    } while (0)
    // ---- cross GOCA-CFAR (fsf:192-213); hits go to an LDS queue so that the S9 work is
    //      spread over the whole workgroup instead of serialising in the lane that owns a range cell
    if (FAST && (RT == 64 || RT == 32)) {   // RT = 32: long-P tiles (LDS cap in the plan)
        // a thread takes 4 adjacent range cells of one Doppler row: every window value comes
        // from float4 LDS reads (17 per 4 cells instead of 20 scalar reads per cell); sums run
        // left to right over each slice like mean()
        constexpr int DL = -(GR + RR), DR = GR + 1;              // window starts rel. to the cell
        constexpr int BL = floor4(DL), BR = floor4(DR);
        constexpr int NL = (DL + 3 + RR - BL + 3) / 4, NR = (DR + 3 + RR - BR + 3) / 4;
        const int lgT = RT == 64 ? 4 : 3;                         // log2 threads per row (RT / 4)
        const int q = threadIdx.x & ((1 << lgT) - 1);
        const int c = hR + 4 * q;                                 // first tile column of the group
        const int r = c0 + c;
        // 16-lane row groups of a wave take rows {0, 2, 1, 3} + 4w: the ds_read_b128 lane groups
        // ({0-3,12-15,20-27}, ... MI355X_MICROARCH.md §LDS) then pair rows 2 apart, 2W = 192
        // floats = 0 mod 64 banks, conflict-free (adjacent rows, W = 96 = 32 mod 64, were 2-way)
        const int rg = threadIdx.x >> lgT;
        const int rgp = lgT == 4 ? (rg & ~3) | ((rg & 1) << 1) | ((rg >> 1) & 1) : rg;
#pragma unroll 1
        for (int v = v0 + rgp; v < v1; v += RSP_THREADS >> lgT) {
            const float* row = S + v * W + c;
            float xl[4 * NL], xr[4 * NR], cv[4];
            f2 lv01 = {0.f, 0.f}, lv23 = {0.f, 0.f}, tv01 = {0.f, 0.f}, tv23 = {0.f, 0.f};   // packed column sums
#pragma unroll
            for (int j = 0; j < NL; ++j) {
                const float4 t = *reinterpret_cast<const float4*>(row + BL + 4 * j);
                xl[4 * j] = t.x; xl[4 * j + 1] = t.y; xl[4 * j + 2] = t.z; xl[4 * j + 3] = t.w;
            }
#pragma unroll
            for (int j = 0; j < NR; ++j) {
                const float4 t = *reinterpret_cast<const float4*>(row + BR + 4 * j);
                xr[4 * j] = t.x; xr[4 * j + 1] = t.y; xr[4 * j + 2] = t.z; xr[4 * j + 3] = t.w;
            }
            {
                const float4 t = *reinterpret_cast<const float4*>(row);
                cv[0] = t.x; cv[1] = t.y; cv[2] = t.z; cv[3] = t.w;
            }
#pragma unroll
            for (int qq = 0; qq < RV; ++qq) {
                const float4 a = *reinterpret_cast<const float4*>(row + (qq - GV - RV) * W);
                const float4 b = *reinterpret_cast<const float4*>(row + (qq + GV + 1) * W);
                lv01 += f2{a.x, a.y};
                lv23 += f2{a.z, a.w};
                tv01 += f2{b.x, b.y};
                tv23 += f2{b.z, b.w};
            }
            const float lv[4] = {lv01.x, lv01.y, lv23.x, lv23.y}, tv[4] = {tv01.x, tv01.y, tv23.x, tv23.y};
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                float lr = 0.f, tr = 0.f;
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
                const float* rowp = S + v * W;
                float lr = 0.f, tr = 0.f, lv = 0.f, tv = 0.f;
                const float* lrp = rowp + c - gR - rR;
                const float* trp = rowp + c + gR + 1;
                const float* lvp = S + (v - gV - rV) * W + c;
                const float* tvp = S + (v + gV + 1) * W + c;
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
    trace_stamp(fp, 2);
    const int n = min(qn[0], K3_QCAP);
    if (n == 0) {
        trace_stamp(fp, 3);
        return;
    }
    if (threadIdx.x == 0) qn[1] = atomicAdd(fp.count[f], n);   // one global reservation per workgroup
    __syncthreads();
    const int base = qn[1];
    for (int i = threadIdx.x; i < n; i += RSP_THREADS) {
        const int idx = base + i;
        if (idx >= g.max_dets) break;
        const int e = queue[i];
        const int v = e >> 16, c = e & 0xFFFF;
        s9_estimate(k, S, W, c0, P, G, Gp, v, c0 + c, pair, MA, MB, &fp.dets[f][idx]);
    }
    if (fp.trace) {
        __syncthreads();
        trace_stamp(fp, 3);
    }
}

// ======================================================================================
// MTD over pulses of a pulse-compressed cube pc[B][P][G] -> rdm[B][P][G] (fsf:131-136)
// ======================================================================================
template <int LGP>
__global__ __launch_bounds__(RSP_THREADS, 2) void k_mtd_cols(Geometry g, DevConsts k, const float2* __restrict__ pc,
                                                        float2* __restrict__ rdm) {
    extern __shared__ __attribute__((aligned(16))) float2 Y[];   // [GT][Ppad] + W_P table
    constexpr int GT = 16;
    float2* twl = Y + GT * g.Ppad;
    if constexpr (LGP > 0)
        for (int i = threadIdx.x; i < tw_total(LGP); i += RSP_THREADS) twl[i] = k.twPp[i];
    const int b = blockIdx.y, gt0 = blockIdx.x * GT;
    const int P = g.P, G = g.G, Ppad = g.Ppad;
    for (int e = threadIdx.x; e < P * GT; e += RSP_THREADS) {
        const int m = e / GT, gl = e - m * GT;
        const int gg = gt0 + gl;
        float2 val = make_float2(0.f, 0.f);
        if (gg < G) {
            val = pc[((size_t)b * P + m) * G + gg];
            val.x *= k.win[m];
            val.y *= k.win[m];
        }
        Y[gl * Ppad + m] = val;
    }
    __syncthreads();
    const int half = P >> 1;
    if constexpr (LGP > 0) {
        StoreLds st{Y};
        fft_passes<LGP, 0, 0, (16 << LGP) / RSP_THREADS, false, 0, RSP_THREADS>(Y, Ppad, GT, twl, st, st);
        for (int e = threadIdx.x; e < P * GT; e += RSP_THREADS) {
            const int v = e / GT, gl = e - v * GT;
            const int gg = gt0 + gl;
            int src = v - half;
            if (src < 0) src += P;
            if (gg < G) rdm[((size_t)b * P + v) * G + gg] = Y[gl * Ppad + src];
        }
    } else {
        for (int e = threadIdx.x; e < P * GT; e += RSP_THREADS) {
            const int v = e / GT, gl = e - v * GT;
            const int gg = gt0 + gl;
            int kk = v - half;
            if (kk < 0) kk += P;
            float2 acc = make_float2(0.f, 0.f);
            int idx = 0;
            for (int p = 0; p < P; ++p) {
                acc = cadd(acc, cmul(Y[gl * Ppad + p], k.twP[idx]));
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
__global__ __launch_bounds__(RSP_THREADS) void k_synth(Geometry g, const double* __restrict__ tx,
                                                     const SynthTarget* __restrict__ tg, int nt, int frame_idx,
                                                     uint64_t seed, double nscale, float2* __restrict__ cube) {
    const size_t total = (size_t)g.P * g.N * g.C;
    const size_t i = (size_t)blockIdx.x * RSP_THREADS + threadIdx.x;
    if (i >= total) return;
    const int m = (int)(i % g.P);
    const size_t rest = i / g.P;
    const int n = (int)(rest % g.N);
    const int c = (int)(rest / g.N);
    const size_t o = (size_t)c * g.cpitch + (size_t)n * g.P + m;   // pitched store offset
    double re = 0.0, im = 0.0;
    for (int t = 0; t < nt; ++t) {
        const int ds = tg[t].delay;
        if (ds > 0 && ds < g.N && n >= ds) {
            const double tr = tx[2 * (n - ds)], ti = tx[2 * (n - ds) + 1];
            double sd, cd, sp, cp;
            sincos(2.0 * M_PI * tg[t].fd_prt * m, &sd, &cd);       // doppler_phase_shift (fsf:58)
            sincos((double)c * tg[t].dphi, &sp, &cp);             // channel phasor (fsf:71-72)
            const double er = tg[t].amp * (tr * cd - ti * sd);     // amplitude * base * doppler
            const double ei = tg[t].amp * (tr * sd + ti * cd);
            re += er * cp - ei * sp;
            im += er * sp + ei * cp;
        }
    }
    // Philox noise (oracle/philox.py documents the stream)
    const uint64_t pairi = (uint64_t)i >> 1;
    uint32_t ctr[4] = {(uint32_t)pairi, (uint32_t)(pairi >> 32), (uint32_t)frame_idx, 0x52535020u};
    rsp_philox10(ctr, (uint32_t)seed, (uint32_t)(seed >> 32));
    const uint32_t xa = (i & 1) ? ctr[2] : ctr[0];
    const uint32_t xb = (i & 1) ? ctr[3] : ctr[1];
    const double ua = ((double)xa + 0.5) * 2.3283064365386963e-10;
    const double ub = ((double)xb + 0.5) * 2.3283064365386963e-10;
    const double rr = sqrt(-2.0 * log(ua));
    double sb, cb;
    sincos(2.0 * M_PI * ub, &sb, &cb);
    re += rr * cb * nscale;
    im += rr * sb * nscale;
    cube[o] = make_float2((float)re, (float)im);
}

}  // namespace

// ---------------------------------------------------------------------------------------
// Dynamic LDS above 64 KiB must be opted in per kernel (gfx950 has 160 KiB per CU).
template <class K>
static hipError_t allow_lds(K kernel, size_t bytes) {
    if (bytes <= 64 * 1024) return hipSuccess;
    return hipFuncSetAttribute(reinterpret_cast<const void*>(kernel), hipFuncAttributeMaxDynamicSharedMemorySize,
                               (int)bytes);
}

template <int BMAX, int CP>
static hipError_t launch_k1_t(const Geometry& g, const DevConsts& k, const FramePtrs& fp, int nf, int mode,
                              hipStream_t s) {
    constexpr int NJ = CP / 4, MB = BMAX <= 8 ? 1 : 2, TPW = (16 / NJ) / MB > 0 ? (16 / NJ) / MB : 1;
    const size_t ldsp = ((size_t)((g.dbg & 8192) ? 1 : 2) * g.B * g.NT * g.Ppad + g.P) * sizeof(float2);
    if (mode == 3 && g.pow2P && g.NT * ((g.P + 31) >> 5) <= (K1_THREADS / 64) * TPW && ldsp <= 160 * 1024 &&
        g.ncu > 0 && !(g.dbg & 4096)) {   // RSP_ABLATE=4096: the non-persistent kernel
        // one FFT size per instantiation keeps the prefetch registers + FFT under 256 VGPRs
        const int grid = std::min(g.ncu, nf * g.ntiles);
#define K1P_LAUNCH(LGP)                                                                                     \
    do {                                                                                                    \
        hipError_t e = allow_lds(k1p_dbf_mtd<BMAX, CP, LGP>, ldsp);                                         \
        if (e != hipSuccess) return e;                                                                      \
        hipLaunchKernelGGL((k1p_dbf_mtd<BMAX, CP, LGP>), dim3(grid), dim3(K1_THREADS), ldsp, s, g, k, fp, nf); \
        return hipGetLastError();                                                                           \
    } while (0)
        switch (g.logP) {
            case 6: K1P_LAUNCH(6);
            case 7: K1P_LAUNCH(7);
            case 8: K1P_LAUNCH(8);
            default: break;
        }
#undef K1P_LAUNCH
    }
    const size_t lds = ((size_t)g.B * g.NT * g.Ppad + g.P) * sizeof(float2);
    hipError_t e = allow_lds(k1_dbf_mtd<BMAX, CP>, lds);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL((k1_dbf_mtd<BMAX, CP>), dim3(g.ntiles, nf), dim3(K1_THREADS), lds, s, g, k, fp, mode);
    return hipGetLastError();
}

template <int BMAX>
static hipError_t launch_k1_b(const Geometry& g, const DevConsts& k, const FramePtrs& fp, int nf, int mode,
                              int ch, hipStream_t s) {
    if (ch <= 8) return launch_k1_t<BMAX, 8>(g, k, fp, nf, mode, s);
    if (ch <= 16) return launch_k1_t<BMAX, 16>(g, k, fp, nf, mode, s);
    return launch_k1_t<BMAX, 32>(g, k, fp, nf, mode, s);
}

hipError_t launch_k1(const Geometry& g, const DevConsts& k, const FramePtrs& fp, int nf, int mode, int,
                     hipStream_t s) {
    if (g.B <= 4) return launch_k1_b<4>(g, k, fp, nf, mode, g.C, s);
    if (g.B <= 8) return launch_k1_b<8>(g, k, fp, nf, mode, g.C, s);
    return launch_k1_b<16>(g, k, fp, nf, mode, g.C, s);
}

hipError_t launch_k2(const Geometry& g, const DevConsts& k, const FramePtrs& fp, int nf, int rows,
                     hipStream_t s) {
    hipError_t e;
    const size_t lds_g = (size_t)(RSP_K2_POINTS + RSP_K2_POINTS / 16) * sizeof(float2);
    const size_t lds_l = (size_t)(K2_LDS_DATA + ((g.dbg & 256) ? K2_LDS_TW : K2_LDS_TW_CMP)) * sizeof(float2);
    // twiddles read in place from global memory (L1/L2), or (dbg 64) copied to LDS; tables in
    // compact rows, or (dbg 256, built so by the plan) full rows.  Default = the fastest
    // measured (profiles/).
#define K2_LAUNCH(TWG, CMP, LDS)                                                                     \
    do {                                                                                             \
        if ((e = allow_lds(k2_pc<TWG, CMP>, LDS)) != hipSuccess) return e;                           \
        if (g.nwg_k2_pow2 > 0)                                                                       \
            hipLaunchKernelGGL((k2_pc<TWG, CMP>), dim3(g.nwg_k2_pow2, nf), dim3(K2_THREADS), LDS, s, g, k, fp, rows); \
    } while (0)
    switch (g.dbg & (64 | 256)) {
        case 0: K2_LAUNCH(true, true, lds_g); break;
        case 64: K2_LAUNCH(false, true, lds_l); break;
        case 256: K2_LAUNCH(true, false, lds_g); break;
        default: K2_LAUNCH(false, false, lds_l); break;
    }
#undef K2_LAUNCH
    if (g.nwg_k2 > g.nwg_k2_pow2) {   // mixed-radix jobs (RSP_K2_MIXED=2): their own 320-thread launch
        const SegDesc& sd = g.segs[g.jobs[g.mix_job0].seg];
        const size_t lds = (size_t)2 * (sd.mixM + (sd.mixM >> K2_SH)) * sizeof(float2);
        const dim3 grid(g.nwg_k2 - g.nwg_k2_pow2, nf);
#define K2M_LAUNCH(M, RA, RB, RC)                                                                    \
    do {                                                                                             \
        if ((e = allow_lds(k2m_pc<M, RA, RB, RC>, lds)) != hipSuccess) return e;                     \
        hipLaunchKernelGGL((k2m_pc<M, RA, RB, RC>), grid, dim3(K2M_THREADS), lds, s, g, k, fp, rows); \
    } while (0)
        switch (sd.mixM) {
            case 640: K2M_LAUNCH(640, 8, 8, 10); break;
            case 1280: K2M_LAUNCH(1280, 16, 8, 10); break;
            default: K2M_LAUNCH(2560, 16, 16, 10); break;
        }
#undef K2M_LAUNCH
    }
    return hipGetLastError();
}

hipError_t launch_k3(const Geometry& g, const DevConsts& k, const FramePtrs& fp, int nf, hipStream_t s) {
    if (g.B < 2 || g.G - 2 * (g.refR + g.guardR) <= 0) return hipSuccess;
    const size_t lds = (size_t)g.P * g.cfar_W * sizeof(float) + (K3_QCAP + 4) * sizeof(int);
    const dim3 grid(k3_ntiles(g) * (g.B - 1) * nf);   // 1-D; k3_cfar remaps it XCD-aware
    hipError_t e;
    if (g.refR == 5 && g.refV == 5 && g.guardR == 10 && g.guardV == 10) {   // the reference's cfar_params (v8:45-46)
        if ((e = allow_lds(k3_cfar<5, 5, 10, 10>, lds)) != hipSuccess) return e;
        hipLaunchKernelGGL((k3_cfar<5, 5, 10, 10>), grid, dim3(RSP_THREADS), lds, s, g, k, fp);
    } else {
        if ((e = allow_lds(k3_cfar<0, 0, 0, 0>, lds)) != hipSuccess) return e;
        hipLaunchKernelGGL((k3_cfar<0, 0, 0, 0>), grid, dim3(RSP_THREADS), lds, s, g, k, fp);
    }
    return hipGetLastError();
}

template <int LGP>
static hipError_t launch_mtd_t(const Geometry& g, const DevConsts& k, const float2* pc, float2* rdm, hipStream_t s) {
    const size_t lds = ((size_t)16 * g.Ppad + g.P) * sizeof(float2);
    hipError_t e = allow_lds(k_mtd_cols<LGP>, lds);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_mtd_cols<LGP>, dim3((g.G + 15) / 16, g.B), dim3(RSP_THREADS), lds, s, g, k, pc, rdm);
    return hipGetLastError();
}

hipError_t launch_mtd_cols(const Geometry& g, const DevConsts& k, const float2* pc, float2* rdm, hipStream_t s) {
    switch (g.pow2P ? g.logP : 0) {
        case 4: return launch_mtd_t<4>(g, k, pc, rdm, s);
        case 5: return launch_mtd_t<5>(g, k, pc, rdm, s);
        case 6: return launch_mtd_t<6>(g, k, pc, rdm, s);
        case 7: return launch_mtd_t<7>(g, k, pc, rdm, s);
        case 8: return launch_mtd_t<8>(g, k, pc, rdm, s);
        case 9: return launch_mtd_t<9>(g, k, pc, rdm, s);
        default: return launch_mtd_t<0>(g, k, pc, rdm, s);
    }
}

hipError_t launch_synth(const Geometry& g, const double* tx, const SynthTarget* tg, int nt, int frame_idx,
                        uint64_t seed, double nscale, float2* cube, hipStream_t s) {
    const size_t total = (size_t)g.P * g.N * g.C;
    const unsigned blocks = (unsigned)((total + RSP_THREADS - 1) / RSP_THREADS);
    hipLaunchKernelGGL(k_synth, dim3(blocks), dim3(RSP_THREADS), 0, s, g, tx, tg, nt, frame_idx, seed, nscale,
                       cube);
    return hipGetLastError();
}
