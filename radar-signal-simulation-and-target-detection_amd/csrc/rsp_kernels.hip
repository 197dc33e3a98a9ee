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
template <bool INV>
__device__ __forceinline__ float2 rot_mi(float2 a) {   // * (-i) forward, * (+i) inverse
    return INV ? make_float2(-a.y, a.x) : make_float2(a.y, -a.x);
}
template <bool INV>
__device__ __forceinline__ float2 twc(float c, float s) {  // exp(-+ i theta) with (c, s) = (cos, sin)
    return make_float2(c, INV ? s : -s);
}

// ---- radix-R DFT kernels in registers -------------------------------------------------
template <int R, bool INV> struct Dft;
template <bool INV> struct Dft<2, INV> {
    static __device__ __forceinline__ void run(float2* a) {
        float2 t = a[0];
        a[0] = cadd(t, a[1]);
        a[1] = csub(t, a[1]);
    }
};
template <bool INV> struct Dft<4, INV> {
    static __device__ __forceinline__ void run(float2* a) {
        float2 t0 = cadd(a[0], a[2]), t1 = csub(a[0], a[2]);
        float2 t2 = cadd(a[1], a[3]), t3 = rot_mi<INV>(csub(a[1], a[3]));
        a[0] = cadd(t0, t2);
        a[2] = csub(t0, t2);
        a[1] = cadd(t1, t3);
        a[3] = csub(t1, t3);
    }
};
template <bool INV> struct Dft<8, INV> {
    static __device__ __forceinline__ void run(float2* a) {
        float2 e[4] = {a[0], a[2], a[4], a[6]};
        float2 o[4] = {a[1], a[3], a[5], a[7]};
        Dft<4, INV>::run(e);
        Dft<4, INV>::run(o);
        const float r = 0.70710678118654752f;
        o[1] = cmul(o[1], twc<INV>(r, r));
        o[2] = rot_mi<INV>(o[2]);
        o[3] = cmul(o[3], twc<INV>(-r, r));
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            a[k] = cadd(e[k], o[k]);
            a[k + 4] = csub(e[k], o[k]);
        }
    }
};
template <bool INV> struct Dft<16, INV> {
    static __device__ __forceinline__ void run(float2* a) {
        float2 e[8], o[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            e[k] = a[2 * k];
            o[k] = a[2 * k + 1];
        }
        Dft<8, INV>::run(e);
        Dft<8, INV>::run(o);
        const float c1 = 0.92387953251128674f, s1 = 0.38268343236508977f, r = 0.70710678118654752f;
        o[1] = cmul(o[1], twc<INV>(c1, s1));
        o[2] = cmul(o[2], twc<INV>(r, r));
        o[3] = cmul(o[3], twc<INV>(s1, c1));
        o[4] = rot_mi<INV>(o[4]);
        o[5] = cmul(o[5], twc<INV>(-s1, c1));
        o[6] = cmul(o[6], twc<INV>(-r, r));
        o[7] = cmul(o[7], twc<INV>(-c1, s1));
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            a[k] = cadd(e[k], o[k]);
            a[k + 8] = csub(e[k], o[k]);
        }
    }
};

template <int R> struct Log2R;
template <> struct Log2R<2> { static constexpr int v = 1; };
template <> struct Log2R<4> { static constexpr int v = 2; };
template <> struct Log2R<8> { static constexpr int v = 3; };
template <> struct Log2R<16> { static constexpr int v = 4; };

// LDS index inside a row: PAD inserts one complex every 16 to break power-of-two strides.
template <bool PAD>
__device__ __forceinline__ int lidx(int i) { return PAD ? i + (i >> 4) : i; }

// Store policies for the Stockham pass output.
struct StoreLds {
    float2* buf; int rs; const float2* H;   // optional pointwise multiply (natural order)
    template <bool PAD>
    __device__ __forceinline__ void put(int row, int o, float2 x) const {
        if (H) x = cmul(x, H[o]);
        buf[row * rs + lidx<PAD>(o)] = x;
    }
};

// One Stockham radix-R pass (Govindaraju et al. formulation) over `nrows` rows of
// length L (= 2^lgL) held in LDS (row stride rs).  Ns = product of earlier radices.
// Reads stride L/R (conflict-light), twiddle W_{Ns R}^{(j mod Ns) r} from the W_L table,
// radix-R DFT, writes positions expand(j, Ns, R) + r Ns.  In place: all reads, barrier,
// all writes, barrier.
template <int R, bool INV, int NB, bool PAD, class St>
__device__ __forceinline__ void sh_pass(float2* buf, int rs, int lgL, int lgNs, int nrows,
                                        const float2* __restrict__ tw, const St& st) {
    constexpr int lgR = Log2R<R>::v;
    const int lgnb = lgL - lgR;
    const int nb = 1 << lgnb;
    const int total = nb * nrows;
    const int Ns = 1 << lgNs;
    const int tid = threadIdx.x;
    float2 v[NB][R];
#pragma unroll
    for (int t = 0; t < NB; ++t) {
        const int beta = tid + t * RSP_THREADS;
        if (beta < total) {
            const int row = beta >> lgnb, j = beta & (nb - 1);
            const int k = j & (Ns - 1);
            const float2* src = buf + row * rs;
            const int step = k << (lgL - lgNs - lgR);
#pragma unroll
            for (int r = 0; r < R; ++r) {
                float2 x = src[lidx<PAD>(j + r * nb)];
                if (r > 0 && lgNs > 0) {
                    float2 w = tw[r * step];
                    if (INV) w.y = -w.y;
                    x = cmul(x, w);
                }
                v[t][r] = x;
            }
        }
    }
    __syncthreads();
#pragma unroll
    for (int t = 0; t < NB; ++t) {
        const int beta = tid + t * RSP_THREADS;
        if (beta < total) {
            const int row = beta >> lgnb, j = beta & (nb - 1);
            const int k = j & (Ns - 1);
            Dft<R, INV>::run(v[t]);
            const int idxD = ((j >> lgNs) << (lgNs + lgR)) + k;
#pragma unroll
            for (int r = 0; r < R; ++r) st.template put<PAD>(row, idxD + r * Ns, v[t][r]);
        }
    }
    __syncthreads();
}

template <int PTS, bool INV, bool PAD, class St>
__device__ __forceinline__ void run_pass(int R, float2* buf, int rs, int lgL, int lgNs, int nrows,
                                         const float2* __restrict__ tw, const St& st) {
    switch (R) {
        case 16: sh_pass<16, INV, (PTS + 15) / 16, PAD>(buf, rs, lgL, lgNs, nrows, tw, st); break;
        case 8: sh_pass<8, INV, (PTS + 7) / 8, PAD>(buf, rs, lgL, lgNs, nrows, tw, st); break;
        case 4: sh_pass<4, INV, (PTS + 3) / 4, PAD>(buf, rs, lgL, lgNs, nrows, tw, st); break;
        default: sh_pass<2, INV, (PTS + 1) / 2, PAD>(buf, rs, lgL, lgNs, nrows, tw, st); break;
    }
}

__device__ __forceinline__ int ilog2(int x) { return 31 - __clz(x); }

// z (compacted Doppler-domain rows) addressing: row (b, v), compacted sample n'.
__device__ __forceinline__ size_t zaddr(const Geometry& g, int b, int v, int np) {
    const int lgNT = ilog2(g.NT);
    return (((size_t)b * g.ntiles + (np >> lgNT)) * g.P + v) * g.NT + (np & (g.NT - 1));
}

// ======================================================================================
// K1: DBF + MTD window + slow-time FFT + fftshift -> compacted rows
// ======================================================================================
template <int BMAX>
__global__ __launch_bounds__(RSP_THREADS, 2) void k1_dbf_mtd(Geometry g, DevConsts k, FramePtrs fp, int mode) {
    extern __shared__ __attribute__((aligned(16))) float2 Y[];   // [B][NT][Ppad]
    const int f = blockIdx.y, tile = blockIdx.x;
    const int B = g.B, C = g.C, P = g.P, NT = g.NT, Ppad = g.Ppad;
    const float2* __restrict__ x = fp.in[f];
    const size_t NP4 = (size_t)g.N * P / 2;   // channel stride in float4 (2 pulses)
    const int halfP = P >> 1;
    const int items = NT * halfP;
    // ---- Phase A: DBF (fsf:93-97) + MTD window (fsf:134), two pulses per thread (16 B loads)
    for (int it = threadIdx.x; it < items; it += RSP_THREADS) {
        const int nl = it / halfP, pp = it - nl * halfP;
        const int n = k.nof[tile * NT + nl];
        float4 acc[BMAX];
#pragma unroll
        for (int b = 0; b < BMAX; ++b) acc[b] = make_float4(0.f, 0.f, 0.f, 0.f);
        if (n >= 0) {
            const float4* __restrict__ src = reinterpret_cast<const float4*>(x + (size_t)n * P) + pp;
            if (mode & 1) {
                for (int c0 = 0; c0 < C; c0 += 8) {
                    float4 xv[8];
#pragma unroll
                    for (int u = 0; u < 8; ++u)
                        xv[u] = (c0 + u < C) ? src[(size_t)(c0 + u) * NP4] : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
                    for (int u = 0; u < 8; ++u) {
                        if (c0 + u < C) {
#pragma unroll
                            for (int b = 0; b < BMAX; ++b) {
                                if (b < B) {
                                    const float2 w = k.Wc[b * C + c0 + u];   // conj(W[b][c])
                                    acc[b].x += xv[u].x * w.x - xv[u].y * w.y;
                                    acc[b].y += xv[u].x * w.y + xv[u].y * w.x;
                                    acc[b].z += xv[u].z * w.x - xv[u].w * w.y;
                                    acc[b].w += xv[u].z * w.y + xv[u].w * w.x;
                                }
                            }
                        }
                    }
                }
            } else {
#pragma unroll
                for (int b = 0; b < BMAX; ++b)
                    if (b < B) acc[b] = src[(size_t)b * NP4];
            }
            if (mode & 2) {
                const float w0 = k.win[2 * pp], w1 = k.win[2 * pp + 1];
#pragma unroll
                for (int b = 0; b < BMAX; ++b) {
                    acc[b].x *= w0; acc[b].y *= w0;
                    acc[b].z *= w1; acc[b].w *= w1;
                }
            }
        }
#pragma unroll
        for (int b = 0; b < BMAX; ++b)
            if (b < B) *reinterpret_cast<float4*>(&Y[(b * NT + nl) * Ppad + 2 * pp]) = acc[b];
    }
    __syncthreads();
    float2* __restrict__ z = fp.z[f];
    const int zslab = P * NT;   // contiguous [P][NT] slab per (b, tile)
    if (!(mode & 2)) {
        for (int e = threadIdx.x; e < B * zslab; e += RSP_THREADS) {
            const int b = e / zslab, rem = e - b * zslab;
            const int v = rem / NT, nl = rem - v * NT;
            z[((size_t)b * g.ntiles + tile) * zslab + rem] = Y[(b * NT + nl) * Ppad + v];
        }
        return;
    }
    const int half = P >> 1;
    if (g.pow2P) {
        // ---- Phase B: P-point FFT of every (b, nl) column (fsf:135)
        const int ncols = B * NT;
        StoreLds st{Y, Ppad, nullptr};
        int lgNs = 0;
        for (int q = 0; q < g.nradP; ++q) {
            const int R = g.radP[q];
            run_pass<32, false, false>(R, Y, Ppad, g.logP, lgNs, ncols, k.twP, st);
            lgNs += ilog2(R);
        }
        // ---- Phase C: fftshift (fsf:135) + coalesced store of the [P][NT] slabs
        for (int e = threadIdx.x; e < B * zslab; e += RSP_THREADS) {
            const int b = e / zslab, rem = e - b * zslab;
            const int v = rem / NT, nl = rem - v * NT;
            int src = v - half;
            if (src < 0) src += P;
            z[((size_t)b * g.ntiles + tile) * zslab + rem] = Y[(b * NT + nl) * Ppad + src];
        }
    } else {
        // non power-of-two P: direct DFT straight to global (O(P^2) per column)
        for (int e = threadIdx.x; e < B * zslab; e += RSP_THREADS) {
            const int b = e / zslab, rem = e - b * zslab;
            const int v = rem / NT, nl = rem - v * NT;
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

// ======================================================================================
// K2: pulse compression of every row (fsf:101-126)
// ======================================================================================
struct StoreRdm {   // last inverse pass: keep outputs i in [Lh-1, Lh-1+V) that map to gates < gend
    float2* rdm; int G; int row0; int rows_total; int Lh1; int g0; int gend;
    template <bool PAD>
    __device__ __forceinline__ void put(int row, int o, float2 x) const {
        const int gg = g0 + o - Lh1;
        const int rho = row0 + row;
        if (o >= Lh1 && gg < gend && rho < rows_total) rdm[(size_t)rho * G + gg] = x;
    }
};

__global__ __launch_bounds__(RSP_THREADS, 2) void k2_pc(Geometry g, DevConsts k, FramePtrs fp, int rows_total) {
    extern __shared__ __attribute__((aligned(16))) float2 L[];
    const int f = blockIdx.y;
    const int wg = blockIdx.x;
    int ji = 0;
    while (ji + 1 < g.njobs && wg >= k.jobs[ji + 1].wg_begin) ++ji;
    const K2Job job = k.jobs[ji];
    const SegDesc& sd = k.segs[job.seg];
    const int rows = sd.rows_per_wg;
    const int row0 = (wg - job.wg_begin) * rows;
    const float2* __restrict__ z = fp.z[f];
    float2* __restrict__ rdm = fp.rdm[f];
    const int P = g.P, G = g.G;
    const int lo = sd.lo, hi = sd.hi, off = sd.off;

    if (sd.type == 1) {
        const int M = sd.M, lgM = sd.logM, Lh1 = sd.Lh - 1;
        const int g0 = sd.ga + job.blk * sd.V;
        const int a = sd.seg_lo + g0 - Lh1;           // sample index of u[0]
        const int rs = M + (M >> 4);
        // load u (masked to the needed window) into padded LDS rows
        for (int e = threadIdx.x; e < rows * M; e += RSP_THREADS) {
            const int rl = e >> lgM, i = e & (M - 1);
            const int rho = row0 + rl;
            const int n = a + i;
            float2 val = make_float2(0.f, 0.f);
            if (rho < rows_total && n >= lo && n <= hi) {
                const int b = rho / P, v = rho - b * P;
                val = z[zaddr(g, b, v, n - lo + off)];
            }
            L[rl * rs + lidx<true>(i)] = val;
        }
        __syncthreads();
        const float2* tw = k.twM + sd.tw_off;
        const float2* H = k.H + sd.H_off;
        int lgNs = 0;
        for (int q = 0; q < sd.nrad; ++q) {                       // forward FFT, last pass x H
            StoreLds st{L, rs, (q == sd.nrad - 1) ? H : nullptr};
            run_pass<16, false, true>(sd.rad[q], L, rs, lgM, lgNs, rows, tw, st);
            lgNs += ilog2(sd.rad[q]);
        }
        lgNs = 0;
        const int gend = min(sd.gb, g0 + sd.V);
        for (int q = 0; q < sd.nrad; ++q) {                       // inverse FFT (1/M folded in H)
            if (q == sd.nrad - 1) {
                StoreRdm st{rdm, G, row0, rows_total, Lh1, g0, gend};
                run_pass<16, true, true>(sd.rad[q], L, rs, lgM, lgNs, rows, tw, st);
            } else {
                StoreLds st{L, rs, nullptr};
                run_pass<16, true, true>(sd.rad[q], L, rs, lgM, lgNs, rows, tw, st);
            }
            lgNs += ilog2(sd.rad[q]);
        }
    } else {
        // direct FIR (narrow segment): filter() + circshift(-fir_delay) (fsf:111-112)
        const int W = hi - lo + 1;
        float* taps = reinterpret_cast<float*>(L + rows * W);
        for (int e = threadIdx.x; e < sd.ntaps; e += RSP_THREADS) taps[e] = k.taps[sd.taps_off + e];
        for (int e = threadIdx.x; e < rows * W; e += RSP_THREADS) {
            const int rl = e / W, i = e - rl * W;
            const int rho = row0 + rl;
            float2 val = make_float2(0.f, 0.f);
            if (rho < rows_total) {
                const int b = rho / P, v = rho - b * P;
                val = z[zaddr(g, b, v, i + off)];
            }
            L[e] = val;
        }
        __syncthreads();
        const int nout = sd.gb - sd.ga;
        for (int e = threadIdx.x; e < rows * nout; e += RSP_THREADS) {
            const int rl = e / nout, gi = e - rl * nout;
            const int rho = row0 + rl;
            if (rho >= rows_total) continue;
            const int gg = sd.ga + gi;
            int kk = (gg + sd.delay) % sd.Ls;
            if (kk < 0) kk += sd.Ls;
            const int nbase = sd.seg_lo + kk;          // sample of tap 0
            const float2* row = L + rl * W;
            float2 acc = make_float2(0.f, 0.f);
            for (int j = 0; j < sd.ntaps; ++j) {
                const int n = nbase - j;
                if (n < lo) break;                      // zero state of filter() / samples before lo
                if (n <= hi) {
                    const float2 xv = row[n - lo];
                    acc.x += taps[j] * xv.x;
                    acc.y += taps[j] * xv.y;
                }
            }
            rdm[(size_t)rho * G + gg] = acc;
        }
    }
}

// ======================================================================================
// K3: GOCA-CFAR on adjacent-beam sums + compaction + S9 estimation
// ======================================================================================
// Peak of MATLAB interp1(...,'spline') (not-a-knot) sampled at step 1/interp over n
// equally spaced points (fsf:257-260, 272-275); returns the first-argmax abscissa.
__device__ double spline_peak(const double* y, int n, int interp) {
    const int nq = (n - 1) * interp + 1;
    double Mv[5] = {0, 0, 0, 0, 0};
    if (n == 5) {
        Mv[1] = y[0] - 2.0 * y[1] + y[2];
        Mv[3] = y[2] - 2.0 * y[3] + y[4];
        Mv[2] = (6.0 * (y[1] - 2.0 * y[2] + y[3]) - Mv[1] - Mv[3]) * 0.25;
        Mv[0] = 2.0 * Mv[1] - Mv[2];
        Mv[4] = 2.0 * Mv[3] - Mv[2];
    }
    double best = -INFINITY, bx = 0.0;
    for (int q = 0; q < nq; ++q) {
        const double xq = (double)q / interp;
        double val;
        if (n == 5) {
            int i = (int)xq;
            if (i > 3) i = 3;
            const double t = xq - i, u = 1.0 - t;
            val = u * y[i] + t * y[i + 1] + ((u * u * u - u) * Mv[i] + (t * t * t - t) * Mv[i + 1]) / 6.0;
        } else if (n == 4) {
            const double d1 = y[1] - y[0], d2 = y[2] - 2.0 * y[1] + y[0];
            const double d3 = y[3] - 3.0 * y[2] + 3.0 * y[1] - y[0];
            val = y[0] + xq * d1 + xq * (xq - 1.0) * 0.5 * d2 + xq * (xq - 1.0) * (xq - 2.0) / 6.0 * d3;
        } else {
            val = y[0] + xq * (y[1] - y[0]) + xq * (xq - 1.0) * 0.5 * (y[2] - 2.0 * y[1] + y[0]);
        }
        if (val > best) {
            best = val;
            bx = xq;
        }
    }
    return bx;
}

__device__ __forceinline__ float cabsf(float2 a) { return sqrtf(a.x * a.x + a.y * a.y); }

__global__ __launch_bounds__(RSP_THREADS) void k3_cfar(Geometry g, DevConsts k, FramePtrs fp) {
    extern __shared__ __attribute__((aligned(16))) float S[];   // [P][W]
    const int f = blockIdx.z, pair = blockIdx.y, tile = blockIdx.x;
    const int P = g.P, G = g.G, W = g.cfar_W, hR = g.cfar_hR;
    const int rR = g.refR, gR = g.guardR, rV = g.refV, gV = g.guardV;
    const int r_begin = rR + gR + tile * g.cfar_RT;
    const int r_end = min(r_begin + g.cfar_RT, G - rR - gR);
    const int c0 = r_begin - hR;
    const float2* __restrict__ A = fp.rdm[f] + (size_t)pair * P * G;
    const float2* __restrict__ Bm = A + (size_t)P * G;
    for (int e = threadIdx.x; e < P * W; e += RSP_THREADS) {
        const int v = e / W, c = e - v * W;
        const int r = c0 + c;
        float val = 0.f;
        if (r >= 0 && r < G) val = cabsf(A[(size_t)v * G + r]) + cabsf(Bm[(size_t)v * G + r]);
        S[e] = val;
    }
    __syncthreads();
    const int v0 = rV + gV, v1 = P - rV - gV;
    const int nr = r_end - r_begin;
    if (v1 <= v0 || nr <= 0) return;
    const float invR = 1.0f / (float)rR, invV = 1.0f / (float)rV;
    const int ncut = (v1 - v0) * nr;
    for (int e = threadIdx.x; e < ncut; e += RSP_THREADS) {
        const int vi = e / nr, ri = e - vi * nr;
        const int v = v0 + vi, r = r_begin + ri;
        const int c = r - c0;
        const float* rowp = S + v * W;
        float lr = 0.f, tr = 0.f, lv = 0.f, tv = 0.f;
        for (int q = 0; q < rR; ++q) {
            lr += rowp[c - gR - rR + q];
            tr += rowp[c + gR + 1 + q];
        }
        for (int q = 0; q < rV; ++q) {
            lv += S[(v - gV - rV + q) * W + c];
            tv += S[(v + gV + 1 + q) * W + c];
        }
        const float nR = fmaxf(lr * invR, tr * invR);   // mean() = sum / n
        const float nV = fmaxf(lv * invV, tv * invV);
        const float thr = g.T * fmaxf(nR, nV);
        const float cut = rowp[c];
        if (cut > thr) {
            const int idx = atomicAdd(fp.count[f], 1);
            if (idx < g.max_dets) {
                // ---- S9 (fsf:237-290)
                double yr[5], yv[5];
                int nrc = 0, rfirst = -1;
                for (int q = -2; q <= 2; ++q) {
                    const int rr = r + q;
                    if (rr >= 0 && rr < G) {
                        if (rfirst < 0) rfirst = rr;
                        yr[nrc++] = (double)rowp[c + q];
                    }
                }
                int nvc = 0, vfirst = -1;
                for (int q = -2; q <= 2; ++q) {
                    const int vv = v + q;
                    if (vv >= 0 && vv < P) {
                        if (vfirst < 0) vfirst = vv;
                        yv[nvc++] = (double)S[vv * W + c];
                    }
                }
                const double rmax = (nrc < 3) ? (double)r : rfirst + spline_peak(yr, nrc, 8);
                const double vmax = (nvc < 3) ? (double)v : vfirst + spline_peak(yv, nvc, 4);
                const double SA = (double)cabsf(A[(size_t)v * G + r]);
                const double SB = (double)cabsf(Bm[(size_t)v * G + r]);
                const double ratio = (SA - SB) / (SA + SB + 2.220446049250313e-16);
                DevDet d;
                d.v_idx = v + 1;
                d.r_idx = r + 1;
                d.pair_idx = pair + 1;
                d.reserved = 0;
                d.amp = (double)cut;
                d.range = k.range_axis[r] + (rmax - r) * k.deltaR;
                d.velocity = k.velocity_axis[v] + (vmax - v) * k.deltaV;
                d.angle = 0.5 * (k.beam_angles[pair] + k.beam_angles[pair + 1]) + k.klut[pair] * ratio;
                fp.dets[f][idx] = d;
            }
        }
    }
}

// ======================================================================================
// MTD over pulses of a pulse-compressed cube pc[B][P][G] -> rdm[B][P][G] (fsf:131-136)
// ======================================================================================
__global__ __launch_bounds__(RSP_THREADS, 2) void k_mtd_cols(Geometry g, DevConsts k, const float2* __restrict__ pc,
                                                        float2* __restrict__ rdm) {
    extern __shared__ __attribute__((aligned(16))) float2 Y[];   // [GT][Ppad]
    const int GT = 16;
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
    if (g.pow2P) {
        StoreLds st{Y, Ppad, nullptr};
        int lgNs = 0;
        for (int q = 0; q < g.nradP; ++q) {
            run_pass<32, false, false>(g.radP[q], Y, Ppad, g.logP, lgNs, GT, k.twP, st);
            lgNs += ilog2(g.radP[q]);
        }
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
__device__ __forceinline__ void philox10(uint32_t c[4], uint32_t k0, uint32_t k1) {
    const uint32_t M0 = 0xD2511F53u, M1 = 0xCD9E8D57u;
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        const uint64_t p0 = (uint64_t)M0 * c[0];
        const uint64_t p1 = (uint64_t)M1 * c[2];
        const uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
        const uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
        const uint32_t n0 = hi1 ^ c[1] ^ k0, n2 = hi0 ^ c[3] ^ k1;
        c[0] = n0; c[1] = lo1; c[2] = n2; c[3] = lo0;
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
}

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
    philox10(ctr, (uint32_t)seed, (uint32_t)(seed >> 32));
    const uint32_t xa = (i & 1) ? ctr[2] : ctr[0];
    const uint32_t xb = (i & 1) ? ctr[3] : ctr[1];
    const double ua = ((double)xa + 0.5) * 2.3283064365386963e-10;
    const double ub = ((double)xb + 0.5) * 2.3283064365386963e-10;
    const double rr = sqrt(-2.0 * log(ua));
    double sb, cb;
    sincos(2.0 * M_PI * ub, &sb, &cb);
    re += rr * cb * nscale;
    im += rr * sb * nscale;
    cube[i] = make_float2((float)re, (float)im);
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

hipError_t launch_k1(const Geometry& g, const DevConsts& k, const FramePtrs& fp, int nf, int mode, int,
                     hipStream_t s) {
    const size_t lds = (size_t)g.B * g.NT * g.Ppad * sizeof(float2);
    dim3 grid(g.ntiles, nf), blk(RSP_THREADS);
    hipError_t e;
    if (g.B <= 4) {
        if ((e = allow_lds(k1_dbf_mtd<4>, lds)) != hipSuccess) return e;
        hipLaunchKernelGGL(k1_dbf_mtd<4>, grid, blk, lds, s, g, k, fp, mode);
    } else if (g.B <= 8) {
        if ((e = allow_lds(k1_dbf_mtd<8>, lds)) != hipSuccess) return e;
        hipLaunchKernelGGL(k1_dbf_mtd<8>, grid, blk, lds, s, g, k, fp, mode);
    } else {
        if ((e = allow_lds(k1_dbf_mtd<16>, lds)) != hipSuccess) return e;
        hipLaunchKernelGGL(k1_dbf_mtd<16>, grid, blk, lds, s, g, k, fp, mode);
    }
    return hipGetLastError();
}

hipError_t launch_k2(const Geometry& g, const DevConsts& k, const FramePtrs& fp, int nf, int rows,
                     hipStream_t s) {
    const size_t lds = (size_t)(RSP_K2_POINTS + RSP_K2_POINTS / 16) * sizeof(float2);
    hipLaunchKernelGGL(k2_pc, dim3(g.nwg_k2, nf), dim3(RSP_THREADS), lds, s, g, k, fp, rows);
    return hipGetLastError();
}

hipError_t launch_k3(const Geometry& g, const DevConsts& k, const FramePtrs& fp, int nf, hipStream_t s) {
    const int ncut_r = g.G - 2 * (g.refR + g.guardR);
    if (g.B < 2 || ncut_r <= 0) return hipSuccess;
    const int tiles = (ncut_r + g.cfar_RT - 1) / g.cfar_RT;
    const size_t lds = (size_t)g.P * g.cfar_W * sizeof(float);
    hipError_t e = allow_lds(k3_cfar, lds);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k3_cfar, dim3(tiles, g.B - 1, nf), dim3(RSP_THREADS), lds, s, g, k, fp);
    return hipGetLastError();
}

hipError_t launch_mtd_cols(const Geometry& g, const DevConsts& k, const float2* pc, float2* rdm, hipStream_t s) {
    const size_t lds = (size_t)16 * g.Ppad * sizeof(float2);
    hipError_t e = allow_lds(k_mtd_cols, lds);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_mtd_cols, dim3((g.G + 15) / 16, g.B), dim3(RSP_THREADS), lds, s, g, k, pc, rdm);
    return hipGetLastError();
}

hipError_t launch_synth(const Geometry& g, const double* tx, const SynthTarget* tg, int nt, int frame_idx,
                        uint64_t seed, double nscale, float2* cube, hipStream_t s) {
    const size_t total = (size_t)g.P * g.N * g.C;
    const unsigned blocks = (unsigned)((total + RSP_THREADS - 1) / RSP_THREADS);
    hipLaunchKernelGGL(k_synth, dim3(blocks), dim3(RSP_THREADS), 0, s, g, tx, tg, nt, frame_idx, seed, nscale,
                       cube);
    return hipGetLastError();
}
