// rsp_music.hip -- MUSIC direction finding on gfx950 (BASELINE config #5).
//
// Reference: MUSIC_1D.m:21-48 and run_music_algorithm.m:22-69.  Per instance (one snapshot
// matrix X [N x K], N <= 64 channels):
//   R = X X^H / K                          (MUSIC_1D.m:28)   k_music_cov   f32 MFMA
//   [EV, D] = eig(R); sort descend          (MUSIC_1D.m:29-33) k_music_eig   Householder + bisection, one wave
//   P = 1 ./ sum(|Q_n^H S1|.^2); dB          (MUSIC_1D.m:35-41) k_music_eig   (same workgroup)
//   findpeaks + top M                       (MUSIC_1D.m:43-48) k_music_eig   (same workgroup)
// plus the synthetic snapshot model of MUSIC_1D.m:21-24 / run_music_algorithm.m:27-39 with the
// Philox streams documented in oracle/music.py (k_music_synth).
//
// Batching: one workgroup per instance (k_music_eig: one wave per instance); BASELINE config
// #5 runs >= 1024 instances per launch so that the 256 CUs are full.
#include "rsp.h"
#include "rsp_internal.h"

#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

int rsp_set_error(int code, const char* fmt, ...);   // rsp_plan.cpp

#define MU_NMAX 64
#define MU_MMAX 8
#define MU_THREADS 256
#define MU_LDA (MU_NMAX + 1)   // LDS row stride (complex) of A and V: column walks hit 2 banks apart
#define MU_SCAN_MAX 4096
#define MU_TAG_SRC 0x4D555341u     // 'MUSA' (oracle/music.py TAG_SRC)
#define MU_TAG_NOISE 0x4D55534Eu   // 'MUSN' (oracle/music.py TAG_NOISE)

namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));

// Complex N(0,1) pair of linear index i of a Philox stream (oracle/philox.py unit_normal_complex).
__device__ __forceinline__ double2 mu_normal(uint64_t i, uint32_t inst, uint64_t seed, uint32_t tag) {
    const uint64_t pr = i >> 1;
    uint32_t c[4] = {(uint32_t)pr, (uint32_t)(pr >> 32), inst, tag};
    rsp_philox10(c, (uint32_t)seed, (uint32_t)(seed >> 32));
    const uint32_t xa = (i & 1) ? c[2] : c[0];
    const uint32_t xb = (i & 1) ? c[3] : c[1];
    const double ua = ((double)xa + 0.5) * 2.3283064365386963e-10;
    const double ub = ((double)xb + 0.5) * 2.3283064365386963e-10;
    const double r = sqrt(-2.0 * log(ua));
    double s, co;
    sincos(2.0 * M_PI * ub, &s, &co);
    return make_double2(r * co, r * s);
}

// ---------------------------------------------------------------------------------------
// Synthetic snapshots (MUSIC_1D.m:21-24, run_music_algorithm.m:27-39), fp64 like MATLAB,
// stored complex64 [inst][K][N] (MATLAB column-major N x K per instance).  Pass 0 measures
// the signal power (awgn 'measured'), pass 1 adds the noise and stores.
// ---------------------------------------------------------------------------------------
#define MU_SYN_KC 128
__device__ __forceinline__ void mu_store(float2* p, double re, double im) { *p = make_float2((float)re, (float)im); }
__device__ __forceinline__ void mu_store(double2* p, double re, double im) { *p = make_double2(re, im); }
// snr_measured: awgn(X, SNR, 'measured') (MUSIC_1D.m:24), the noise scale follows from pass 0;
// otherwise nsc_fixed = sqrt(noise_power / 2) (run_music_algorithm.m:35-36) and pass 0 is skipped.
// CX: the plan's snapshot type (double2: complex double, MATLAB's; float2: complex single).
template <class CX>
__global__ __launch_bounds__(MU_THREADS) void k_music_synth(int N, int K, int M, int inst0, uint64_t seed,
                                                          const double2* __restrict__ Ssrc, const double* __restrict__ amp,
                                                          int complex_src, int snr_measured, double snr_db,
                                                          double nsc_fixed, CX* __restrict__ X) {
    __shared__ double2 al[MU_MMAX][MU_SYN_KC];
    __shared__ double2 Sl[MU_MMAX][MU_NMAX];
    __shared__ double red[MU_THREADS];
    const int tid = threadIdx.x;
    const uint32_t inst = (uint32_t)(inst0 + blockIdx.x);
    CX* __restrict__ Xi = X + (size_t)blockIdx.x * K * N;
    for (int e = tid; e < M * N; e += MU_THREADS) Sl[e / N][e % N] = Ssrc[e];
    double nsc = nsc_fixed;
    for (int pass = snr_measured ? 0 : 1; pass < 2; ++pass) {
        double psum = 0.0;
        for (int k0 = 0; k0 < K; k0 += MU_SYN_KC) {
            const int kc = min(MU_SYN_KC, K - k0);
            __syncthreads();
            for (int e = tid; e < M * kc; e += MU_THREADS) {   // Alpha(m, k): stream index m + M k
                const int kk = e / M, m = e - kk * M;
                const double2 z = mu_normal((uint64_t)m + (uint64_t)M * (k0 + kk), inst, seed, MU_TAG_SRC);
                al[m][kk] = complex_src ? make_double2(z.x * M_SQRT1_2 * amp[m], z.y * M_SQRT1_2 * amp[m])
                                        : make_double2(z.x * amp[m], 0.0);
            }
            __syncthreads();
            for (int e = tid; e < N * kc; e += MU_THREADS) {
                const int kk = e / N, c = e - kk * N;
                double xr = 0.0, xi = 0.0;
                for (int m = 0; m < M; ++m) {   // X = S * Alpha (MUSIC_1D.m:23)
                    const double2 sv = Sl[m][c], a = al[m][kk];
                    xr += sv.x * a.x - sv.y * a.y;
                    xi += sv.x * a.y + sv.y * a.x;
                }
                if (pass == 0) {
                    psum += xr * xr + xi * xi;
                } else {   // noise: stream index c + N k
                    const uint64_t lin = (uint64_t)c + (uint64_t)N * (k0 + kk);
                    const double2 z = mu_normal(lin, inst, seed, MU_TAG_NOISE);
                    mu_store(Xi + lin, xr + nsc * z.x, xi + nsc * z.y);
                }
            }
        }
        if (pass == 0) {   // noise power = mean|X|^2 / 10^(SNR/10)
            red[tid] = psum;
            __syncthreads();
            for (int h = MU_THREADS / 2; h > 0; h >>= 1) {
                if (tid < h) red[tid] += red[tid + h];
                __syncthreads();
            }
            nsc = sqrt(red[0] / ((double)N * K) / pow(10.0, snr_db / 10.0) / 2.0);
        }
    }
}

// ---------------------------------------------------------------------------------------
// R = X X^H / K on the f32 matrix cores (MUSIC_1D.m:28).  One workgroup (4 waves) per
// instance, split-K over the waves (4-snapshot steps interleaved, so the waves stream adjacent
// 2 KB blocks).  Lane l loads the 4 consecutive channels 4(l&15)..+3 of snapshot 4s + (l>>4):
// 32 B per lane, 512 B per snapshot.  Channel 4r + I is row r of "virtual block" I, so the
// same register is the A operand (A[r][kk] = x_I) and the B operand (B[kk][r] = x_I) of
// v_mfma_f32_16x16x4_f32, and tile (I, J) = sum_k x_I x_J^H holds R[4r+I][4s+J].
// Hermitian: only the 10 tiles I <= J are accumulated (4 MFMAs each per step:
// Re += xr xr' + xi xi', Im += xi xr' - xr xi'); the rest is mirrored at the store.
// ---------------------------------------------------------------------------------------
template <bool VEC4>
__global__ __launch_bounds__(MU_THREADS) void k_music_cov(int N, int K, const float2* __restrict__ X,
                                                        float2* __restrict__ R) {
    __shared__ float red[10][2][256];   // per tile, Re/Im, D[i][j] row-major
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int r = lane & 15, kk = lane >> 4;
    const float2* __restrict__ Xi = X + (size_t)blockIdx.x * K * N;
    f32x4 ar[10], ai[10];
#pragma unroll
    for (int t = 0; t < 10; ++t) {
        ar[t] = f32x4{0.f, 0.f, 0.f, 0.f};
        ai[t] = ar[t];
    }
    const int nsteps = (K + 3) >> 2;
    auto load = [&](int s, float (&xr)[4], float (&xi)[4]) {
        const int k = 4 * s + kk;
        const int c0 = 4 * r;
        if (VEC4) {
            float4 u = make_float4(0.f, 0.f, 0.f, 0.f), v = u;
            if (k < K && c0 < N) {
                const float4* p = reinterpret_cast<const float4*>(Xi + (size_t)k * N + c0);
                u = p[0];
                v = p[1];
            }
            xr[0] = u.x; xi[0] = u.y; xr[1] = u.z; xi[1] = u.w;
            xr[2] = v.x; xi[2] = v.y; xr[3] = v.z; xi[3] = v.w;
        } else {
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                float2 x = make_float2(0.f, 0.f);
                if (k < K && c0 + i < N) x = Xi[(size_t)k * N + c0 + i];
                xr[i] = x.x;
                xi[i] = x.y;
            }
        }
    };
    auto step = [&](const float (&xr)[4], const float (&xi)[4]) {
        float nr[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) nr[i] = -xr[i];
        int t = 0;
#pragma unroll
        for (int I = 0; I < 4; ++I)
#pragma unroll
            for (int J = I; J < 4; ++J, ++t) {
                ar[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(xr[I], xr[J], ar[t], 0, 0, 0);
                ar[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(xi[I], xi[J], ar[t], 0, 0, 0);
                ai[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(xi[I], xr[J], ai[t], 0, 0, 0);
                ai[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(nr[I], xi[J], ai[t], 0, 0, 0);
            }
    };
    // software pipeline: the loads of step s + 8 are in flight while step s computes
    float xr0[4], xi0[4], xr1[4], xi1[4];
    int s = w;
    if (s < nsteps) load(s, xr0, xi0);
    if (s + 4 < nsteps) load(s + 4, xr1, xi1);
    for (; s + 4 < nsteps; s += 8) {
        step(xr0, xi0);
        if (s + 8 < nsteps) load(s + 8, xr0, xi0);
        step(xr1, xi1);
        if (s + 12 < nsteps) load(s + 12, xr1, xi1);
    }
    if (s < nsteps) step(xr0, xi0);
    // ordered cross-wave sum (deterministic): wave 0 stores, waves 1..3 add in turn
    for (int ww = 0; ww < 4; ++ww) {
        if (w == ww) {
#pragma unroll
            for (int t = 0; t < 10; ++t)
#pragma unroll
                for (int v = 0; v < 4; ++v) {
                    const int e = (4 * kk + v) * 16 + r;   // D row 4(l>>4)+v, column l&15
                    if (ww == 0) {
                        red[t][0][e] = ar[t][v];
                        red[t][1][e] = ai[t][v];
                    } else {
                        red[t][0][e] += ar[t][v];
                        red[t][1][e] += ai[t][v];
                    }
                }
        }
        __syncthreads();
    }
    // R[inst] column-major with leading dimension 64: R(a, b) at a + 64 b
    float2* __restrict__ Ri = R + (size_t)blockIdx.x * MU_NMAX * MU_NMAX;
    const float invK = 1.0f / (float)K;
    int t = 0;
    for (int I = 0; I < 4; ++I)
        for (int J = I; J < 4; ++J, ++t) {
            const int i = tid >> 4, j = tid & 15;
            const int a = 4 * i + I, b = 4 * j + J;
            const float re = red[t][0][tid] * invK, im = red[t][1][tid] * invK;
            if (a < N && b < N) {
                Ri[a + MU_NMAX * b] = make_float2(re, im);
                if (I != J) Ri[b + MU_NMAX * a] = make_float2(re, -im);
            }
        }
}

// ---------------------------------------------------------------------------------------
// eig + MUSIC spectrum + findpeaks (MUSIC_1D.m:29-48): ONE WAVE PER INSTANCE, fp32 in LDS.
// Lane i owns matrix column i (N <= 64): every LDS access of A walks a row, so the 64 lanes
// touch 64 consecutive complex words (no bank conflicts); cross-lane operands come from
// v_readlane and DPP reductions, so no phase needs more than a one-wave barrier.
//  1. Householder reduction of the Hermitian R to a real symmetric tridiagonal T = Q^H R Q
//     (LAPACK zhetd2, lower: H_k = I - tau_k v_k v_k^H, beta_k real).  Column k of A is
//     conj(row k); v_k is kept in row k (columns k+1..), which is dead after step k.
//  2. All N eigenvalues of T by Sturm-count bisection, lane t -> t-th smallest (EVA,
//     MUSIC_1D.m:29-31, sorted descending).
//  3. The M signal eigenvectors of T by block inverse iteration (partial-pivot tridiagonal
//     LU as LAPACK dlagtf/dlagts, lane j = vector j, 3 solves with Gram-Schmidt after each),
//     then q_j = H_0 ... H_{n-2} y_j (lane = component).
//  4. sum_j |Q_n^H a|^2 (MUSIC_1D.m:37) = a^H (I - Q_s Q_s^H) a for the unitary [Q_s Q_n],
//     evaluated as |a - Q_s (Q_s^H a)|^2 (no cancellation against |a|^2 = N), lane = angle.
//  5. P = 1 / den, P_dB = 10 log10(P / max P), findpeaks + the M largest (MUSIC_1D.m:37-47).
// Dynamic LDS per wave: A [64][64] complex | tau [64] complex | d, e^2, lambda, e [64] |
// LU + y [5][64][M] (vector fastest) | Q_s [M][64] complex | (v, w) [64][2]; den(s) overlays A.
// ---------------------------------------------------------------------------------------
__device__ __forceinline__ float2 cm(float2 a, float2 b) { return make_float2(a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x); }
__device__ __forceinline__ float2 cmc(float2 a, float2 b) {   // conj(a) * b
    return make_float2(a.x * b.x + a.y * b.y, a.x * b.y - a.y * b.x);
}
__device__ __forceinline__ float2 cadd2(float2 a, float2 b) { return make_float2(a.x + b.x, a.y + b.y); }
__device__ __forceinline__ float2 csub2(float2 a, float2 b) { return make_float2(a.x - b.x, a.y - b.y); }
__device__ __forceinline__ float2 csc(float s, float2 a) { return make_float2(s * a.x, s * a.y); }
__device__ __forceinline__ float2 cconj(float2 a) { return make_float2(a.x, -a.y); }

#define MU_DPP(v, ctrl) __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), (ctrl), 0xF, 0xF, false))
__device__ __forceinline__ float rdl(float v, int l) { return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l)); }
__device__ __forceinline__ float2 rdl2(float2 v, int l) { return make_float2(rdl(v.x, l), rdl(v.y, l)); }
// Sum / max over the 64 lanes, result uniform: DPP butterflies inside each row of 16 lanes
// (quad_perm xor 1, xor 2, half-mirror, mirror), then the four row values by readlane.
__device__ __forceinline__ float wsum(float v) {
    v += MU_DPP(v, 0xB1);
    v += MU_DPP(v, 0x4E);
    v += MU_DPP(v, 0x141);
    v += MU_DPP(v, 0x140);
    return (rdl(v, 0) + rdl(v, 16)) + (rdl(v, 32) + rdl(v, 48));
}
__device__ __forceinline__ float wmax(float v) {
    v = fmaxf(v, MU_DPP(v, 0xB1));
    v = fmaxf(v, MU_DPP(v, 0x4E));
    v = fmaxf(v, MU_DPP(v, 0x141));
    v = fmaxf(v, MU_DPP(v, 0x140));
    return fmaxf(fmaxf(rdl(v, 0), rdl(v, 16)), fmaxf(rdl(v, 32), rdl(v, 48)));
}
__device__ __forceinline__ int wmin_i(int v) {
#define MU_DPPI(x, ctrl) __builtin_amdgcn_update_dpp(0, (x), (ctrl), 0xF, 0xF, false)
    v = min(v, MU_DPPI(v, 0xB1));
    v = min(v, MU_DPPI(v, 0x4E));
    v = min(v, MU_DPPI(v, 0x141));
    v = min(v, MU_DPPI(v, 0x140));
#undef MU_DPPI
    return min(min(__builtin_amdgcn_readlane(v, 0), __builtin_amdgcn_readlane(v, 16)),
               min(__builtin_amdgcn_readlane(v, 32), __builtin_amdgcn_readlane(v, 48)));
}

#define MU_ITER 3            // inverse-iteration solves per signal vector
#define MU_SPW (MU_SCAN_MAX / 64)

__host__ __device__ constexpr size_t mu_eig_lds_bytes(int M) {
    return (size_t)MU_NMAX * MU_NMAX * 8 + MU_NMAX * 8 + 4 * MU_NMAX * 4 + (size_t)5 * M * MU_NMAX * 4 +
           (size_t)M * MU_NMAX * 8 + MU_NMAX * 16;
}

template <int M>   // signal subspace dimension (compile time: the M-vector loops unroll exactly)
__global__ __launch_bounds__(64) void k_music_eig(int N, int S, const float2* __restrict__ R,
                                                const float2* __restrict__ S1T, int Spad, float* __restrict__ spec_db,
                                                float* __restrict__ eig_out, int* __restrict__ peaks_out,
                                                unsigned long long* __restrict__ trace) {
    // trace (diagnostic, RSP_MUSIC_TRACE=1): s_memrealtime at the phase boundaries
#define MU_STAMP(i) \
    if (trace && threadIdx.x == 0) trace[(size_t)blockIdx.x * 8 + (i)] = wall_clock64()
    MU_STAMP(0);
    extern __shared__ __attribute__((aligned(16))) float2 lds[];
    float2* A = lds;                                  // A(j, i) at A[j * 64 + i]
    float2* taus = A + MU_NMAX * MU_NMAX;
    float* dd = reinterpret_cast<float*>(taus + MU_NMAX);
    float* e2 = dd + MU_NMAX;                         // e_k^2
    float* lam = e2 + MU_NMAX;                        // ascending eigenvalues
    float* ee = lam + MU_NMAX;                        // e_k = beta_k (signed)
    float* lu = ee + MU_NMAX;                        // [5][64][M]: U diag, U super 1, U super 2, mult, y
    float2* Qs = reinterpret_cast<float2*>(lu + 5 * MU_NMAX * M);   // [M][64]
    float2* vw = Qs + M * MU_NMAX;                    // [64][2]: (v_j, w_j) of the current step
    const int lane = threadIdx.x;
    const int n = N;
    const bool live = lane < n;
    const float2 z2 = make_float2(0.f, 0.f);
    {   // A(j, i) = conj(R(i, j)): R column-major ld 64, lane i reads R(i, j) (coalesced)
        const float2* __restrict__ Ri = R + (size_t)blockIdx.x * MU_NMAX * MU_NMAX;
        for (int j = 0; j < n; ++j) A[j * MU_NMAX + lane] = live ? cconj(Ri[lane + MU_NMAX * j]) : z2;
        for (int j = n; j < ((n + 7) & ~7); ++j) A[j * MU_NMAX + lane] = z2;   // chunk padding rows
    }
    const int nr = (n + 7) & ~7;
    __syncthreads();
    // ---- 1. tridiagonalisation
    for (int k = 0; k < n - 1; ++k) {
        const float2 x = cconj(A[k * MU_NMAX + lane]);     // x_i = A(i, k), i > k
        const float xn2 = wsum(lane >= k + 2 && live ? x.x * x.x + x.y * x.y : 0.f);
        const float2 al = rdl2(x, k + 1);
        float2 tau = z2, scale = z2;
        float beta = al.x;
        if (xn2 > 0.f || al.y != 0.f) {   // zlarfg (uniform)
            beta = -copysignf(sqrtf(al.x * al.x + al.y * al.y + xn2), al.x);
            tau = make_float2((beta - al.x) / beta, -al.y / beta);
            const float2 dn = make_float2(al.x - beta, al.y);
            const float q = 1.f / (dn.x * dn.x + dn.y * dn.y);
            scale = make_float2(dn.x * q, -dn.y * q);
        }
        if (lane == k) {
            dd[k] = x.x;          // A(k, k) (real)
            e2[k] = beta * beta;
            ee[k] = beta;
            taus[k] = tau;
        }
        const float2 v = lane == k + 1 ? make_float2(1.f, 0.f) : (lane >= k + 2 && live ? cm(x, scale) : z2);
        A[k * MU_NMAX + lane] = v;                           // v_k kept in row k
        if (tau.x == 0.f && tau.y == 0.f) continue;
        // p_i = tau sum_j A(i, j) v_j = tau sum_j conj(A(j, i)) v_j.  Rows in chunks of 8 from
        // (k+1) & ~7 (v_j = w_j = 0 for j <= k and j >= n, padding rows are zero), v_j and w_j
        // read back as LDS broadcasts ((v_j, w_j) interleaved in vw[]); 4 partial sums so the
        // complex FMAs do not form one dependent chain.  (Holding the whole column in registers
        // measured slower: the unrolled kernel outgrew the instruction cache.)
        vw[2 * lane] = v;
        __builtin_amdgcn_wave_barrier();
        const int j0 = (k + 1) & ~7;
        float2 acc[4] = {z2, z2, z2, z2};
        for (int jc = j0; jc < nr; jc += 8) {
            float2 a[8];
            float4 b[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) a[u] = A[(jc + u) * MU_NMAX + lane];
#pragma unroll
            for (int u = 0; u < 8; ++u) b[u] = *reinterpret_cast<const float4*>(vw + 2 * (jc + u));
#pragma unroll
            for (int u = 0; u < 8; ++u) acc[u & 3] = cadd2(acc[u & 3], cmc(a[u], make_float2(b[u].x, b[u].y)));
        }
        const bool act = lane > k && live;
        const float2 p = act ? cm(tau, cadd2(cadd2(acc[0], acc[1]), cadd2(acc[2], acc[3]))) : z2;
        const float2 pv = cmc(p, v);
        const float2 alpha = csc(-0.5f, cm(tau, make_float2(wsum(pv.x), wsum(pv.y))));
        const float2 w = act ? cadd2(p, cm(alpha, v)) : z2;
        vw[2 * lane + 1] = w;
        __builtin_amdgcn_wave_barrier();
        const float2 cw = cconj(w), cv = cconj(v);
        // A(j, i) -= v_j conj(w_i) + w_j conj(v_i); lanes and rows outside k+1..n-1 have
        // v = w = 0 and rewrite their value
        for (int jc = j0; jc < nr; jc += 8) {
            float2 a[8];
            float4 b[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) a[u] = A[(jc + u) * MU_NMAX + lane];
#pragma unroll
            for (int u = 0; u < 8; ++u) b[u] = *reinterpret_cast<const float4*>(vw + 2 * (jc + u));
#pragma unroll
            for (int u = 0; u < 8; ++u)
                A[(jc + u) * MU_NMAX + lane] =
                    csub2(a[u], cadd2(cm(make_float2(b[u].x, b[u].y), cw), cm(make_float2(b[u].z, b[u].w), cv)));
        }
    }
    if (lane == n - 1) dd[n - 1] = A[(n - 1) * MU_NMAX + n - 1].x;
    __syncthreads();
    MU_STAMP(1);
    // ---- 2. eigenvalues by bisection (lane t -> t-th smallest)
    {
        float glo = 3.4e38f, ghi = -3.4e38f;
        for (int i = 0; i < n; ++i) {   // Gershgorin
            const float r = (i > 0 ? sqrtf(e2[i - 1]) : 0.f) + (i < n - 1 ? sqrtf(e2[i]) : 0.f);
            glo = fminf(glo, dd[i] - r);
            ghi = fmaxf(ghi, dd[i] + r);
        }
        const float tn = fmaxf(fabsf(glo), fabsf(ghi));
        const float pivmin = 1e-30f * fmaxf(1.f, tn * tn);
        float lo = glo - 1e-6f * tn - pivmin, hi = ghi + 1e-6f * tn + pivmin;
        for (int it = 0; it < 64; ++it) {
            const bool go = live && hi - lo > 2.4e-7f * fmaxf(fabsf(lo), fabsf(hi)) + pivmin;
            if (!__builtin_amdgcn_ballot_w64(go)) break;
            const float mid = 0.5f * (lo + hi);
            int cnt = 0;
            float q = dd[0] - mid;
            if (fabsf(q) < pivmin) q = -pivmin;
            cnt += q < 0.f;
#pragma unroll 8
            for (int i = 1; i < n; ++i) {
                q = (dd[i] - mid) - e2[i - 1] * __builtin_amdgcn_rcpf(q);
                if (fabsf(q) < pivmin) q = -pivmin;
                cnt += q < 0.f;
            }
            if (go) {
                if (cnt > lane) hi = mid; else lo = mid;
            }
        }
        const float l = 0.5f * (lo + hi);
        if (live) {
            lam[lane] = l;
            eig_out[(size_t)blockIdx.x * N + (n - 1 - lane)] = l;   // descending (MUSIC_1D.m:31)
        }
    }
    __syncthreads();
    MU_STAMP(2);
    // ---- 3. signal eigenvectors of T: block inverse iteration (lane j = vector j)
    float tnorm = 0.f;
    for (int i = 0; i < n; ++i)
        tnorm = fmaxf(tnorm, fabsf(dd[i]) + (i > 0 ? sqrtf(e2[i - 1]) : 0.f) + (i < n - 1 ? sqrtf(e2[i]) : 0.f));
    const float ptol = 1.2e-7f * tnorm + 1e-30f;
#define LU(arr, i) lu[((arr) * MU_NMAX + (i)) * M + lane]
    unsigned long long swp = 0ull;
    if (lane < M) {   // dlagtf on T - lambda_j I; carried values in registers, factors to LDS
        const float lj = lam[n - 1 - lane];
        float ak = dd[0] - lj;                                // current diagonal
        float bk = n > 1 ? ee[0] : 0.f;                       // current super 1 (= e_k)
        for (int k = 0; k < n - 1; ++k) {
            const float ck = ee[k];                           // sub-diagonal e_k
            const float an = dd[k + 1] - lj;                  // next diagonal
            const float bn = k < n - 2 ? ee[k + 1] : 0.f;
            if (fabsf(ak) >= fabsf(ck)) {
                const float a0 = fabsf(ak) < ptol ? copysignf(ptol, ak) : ak;
                const float mult = ck / a0;
                LU(0, k) = a0; LU(1, k) = bk; LU(2, k) = 0.f; LU(3, k) = mult;
                ak = an - mult * bk;
                bk = bn;
            } else {
                swp |= 1ull << k;
                const float mult = ak / ck;
                LU(0, k) = ck; LU(1, k) = an; LU(2, k) = bn; LU(3, k) = mult;
                ak = bk - mult * an;
                bk = -mult * bn;
            }
        }
        LU(0, n - 1) = fabsf(ak) < ptol ? copysignf(ptol, ak) : ak;
        for (int i = 0; i < n; ++i) LU(4, i) = 1.f + 0.0625f * (float)((i * 37 + lane * 11) % 17);   // start
    }
    for (int it = 0; it < MU_ITER; ++it) {
        if (lane < M) {   // dlagts: forward with the interchanges, then U back-substitution
            float yk = LU(4, 0);
            for (int k = 0; k < n - 1; ++k) {
                const float yn = LU(4, k + 1), mult = LU(3, k);
                if (swp >> k & 1ull) {
                    LU(4, k) = yn;
                    yk = yk - mult * yn;
                } else {
                    LU(4, k) = yk;
                    yk = yn - mult * yk;
                }
            }
            float y1 = yk / LU(0, n - 1), y2 = 0.f;
            LU(4, n - 1) = y1;
            for (int k = n - 2; k >= 0; --k) {
                const float yk2 = (LU(4, k) - LU(1, k) * y1 - LU(2, k) * y2) / LU(0, k);
                LU(4, k) = yk2;
                y2 = y1;
                y1 = yk2;
            }
        }
        __syncthreads();
        for (int j = 0; j < M; ++j) {   // modified Gram-Schmidt (lane = component)
            float yj = live ? lu[(4 * MU_NMAX + lane) * M + j] : 0.f;
            for (int i = 0; i < j; ++i) {
                const float yi = live ? lu[(4 * MU_NMAX + lane) * M + i] : 0.f;
                yj -= wsum(yi * yj) * yi;
            }
            yj *= rsqrtf(wsum(yj * yj));
            if (live) lu[(4 * MU_NMAX + lane) * M + j] = yj;
            __syncthreads();
        }
    }
#undef LU
    MU_STAMP(3);
    // q_j = H_0 H_1 ... H_{n-2} y_j (lane = component; the M vectors advance together)
    {
        float2 y[M];
#pragma unroll
        for (int j = 0; j < M; ++j)
            y[j] = make_float2(j < M && live ? lu[(4 * MU_NMAX + lane) * M + j] : 0.f, 0.f);
        for (int k = n - 2; k >= 0; --k) {
            const float2 tau = taus[k];
            const float2 v = lane == k + 1 ? make_float2(1.f, 0.f) : (lane > k + 1 && live ? A[k * MU_NMAX + lane] : z2);
#pragma unroll
            for (int j = 0; j < M; ++j) {
                if (j < M) {
                    const float2 pr = cmc(v, y[j]);
                    const float2 dot = make_float2(wsum(pr.x), wsum(pr.y));
                    y[j] = csub2(y[j], cm(tau, cm(v, dot)));
                }
            }
        }
#pragma unroll
        for (int j = 0; j < M; ++j)
            if (j < M) Qs[j * MU_NMAX + lane] = y[j];
    }
    __syncthreads();
    MU_STAMP(4);
    // ---- 4. den(s) = |a(s) - Q_s Q_s^H a(s)|^2, lane = angle (den overlays A)
    float* den = reinterpret_cast<float*>(A);
    // (the lane's 64 steering values are loaded at once and kept for both passes; rows c >= N
    // of S1T and of Q_s are zero)
    for (int s = lane; s < S; s += 64) {
        float2 a[MU_NMAX];
#pragma unroll
        for (int c = 0; c < MU_NMAX; ++c) a[c] = S1T[(size_t)c * Spad + s];
        float2 cf[M];
#pragma unroll
        for (int m = 0; m < M; ++m) cf[m] = z2;
#pragma unroll
        for (int c = 0; c < MU_NMAX; c += 2)
#pragma unroll
            for (int m = 0; m < M; ++m)
                if (m < M) {
                    const float4 q = *reinterpret_cast<const float4*>(Qs + m * MU_NMAX + c);
                    cf[m] = cadd2(cf[m], cmc(make_float2(q.x, q.y), a[c]));
                    cf[m] = cadd2(cf[m], cmc(make_float2(q.z, q.w), a[c + 1]));
                }
        float r2 = 0.f;
#pragma unroll
        for (int c = 0; c < MU_NMAX; c += 2) {
            float2 r0 = a[c], r1 = a[c + 1];
#pragma unroll
            for (int m = 0; m < M; ++m)
                if (m < M) {
                    const float4 q = *reinterpret_cast<const float4*>(Qs + m * MU_NMAX + c);
                    r0 = csub2(r0, cm(make_float2(q.x, q.y), cf[m]));
                    r1 = csub2(r1, cm(make_float2(q.z, q.w), cf[m]));
                }
            r2 += r0.x * r0.x + r0.y * r0.y;
            r2 += r1.x * r1.x + r1.y * r1.y;
        }
        den[s] = r2;
    }
    __syncthreads();
    MU_STAMP(5);
    // ---- 5. P = 1 ./ den, P_dB = 10 log10(P / max P) (MUSIC_1D.m:37-41)
    float pm = 0.f;
    for (int s = lane; s < S; s += 64) pm = fmaxf(pm, 1.f / den[s]);
    const float pmax = wmax(pm);
    float* __restrict__ out = spec_db + (size_t)blockIdx.x * S;
    for (int s = lane; s < S; s += 64) {
        const float db = 10.f * log10f((1.f / den[s]) / pmax);
        den[s] = db;
        out[s] = db;
    }
    __syncthreads();
    // findpeaks (MUSIC_1D.m:43): s is a peak iff it starts a run of equal values entered by a
    // strict rise and left by a strict fall (ends excluded); then the M largest, ties to the
    // lower index (stable sort 'descend', :44-47)
    unsigned long long pkm = 0ull;   // bit t: s = lane + 64 t is a peak
    int npk = 0;
    for (int t = 0; t * 64 < S; ++t) {
        const int s = lane + 64 * t;
        bool pk = false;
        if (s >= 1 && s < S - 1 && den[s] > den[s - 1]) {
            int u = s + 1;
            while (u < S && den[u] == den[s]) ++u;
            pk = u < S && den[u] < den[s];
        }
        if (pk) pkm |= 1ull << t;
        npk += __popcll(__builtin_amdgcn_ballot_w64(pk));
    }
    int* po = peaks_out + (size_t)blockIdx.x * (MU_MMAX + 1);
    if (lane == 0) po[0] = npk;
    for (int r = 0; r < MU_MMAX; ++r) {
        int sel = 0;
        if (r < M) {
            float bv = -3.4e38f;
            int bs = 1 << 30;
            for (int t = 0; t * 64 < S; ++t)
                if (pkm >> t & 1ull) {
                    const int s = lane + 64 * t;
                    if (den[s] > bv) { bv = den[s]; bs = s; }   // t ascending: ties keep the lower s
                }
            const float gv = wmax(bv);
            const int gs = wmin_i(bv == gv ? bs : (1 << 30));
            if (gs < (1 << 30)) {
                sel = gs + 1;
                if ((gs & 63) == lane) pkm &= ~(1ull << (gs >> 6));
            }
        }
        if (lane == 0) po[1 + r] = sel;
    }
    MU_STAMP(6);
#undef MU_STAMP
}

// =======================================================================================
// Complex double (MATLAB's arithmetic, MUSIC_1D.m:28-48 in double): the default precision.
// =======================================================================================
typedef double f64x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ double2 zm(double2 a, double2 b) { return make_double2(a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x); }
__device__ __forceinline__ double2 zmc(double2 a, double2 b) {   // conj(a) * b
    return make_double2(a.x * b.x + a.y * b.y, a.x * b.y - a.y * b.x);
}
__device__ __forceinline__ double2 zadd(double2 a, double2 b) { return make_double2(a.x + b.x, a.y + b.y); }
__device__ __forceinline__ double2 zsub(double2 a, double2 b) { return make_double2(a.x - b.x, a.y - b.y); }
__device__ __forceinline__ double2 zsc(double s, double2 a) { return make_double2(s * a.x, s * a.y); }
__device__ __forceinline__ double2 zconj(double2 a) { return make_double2(a.x, -a.y); }

// DPP moves of a double (two 32-bit halves), and the quad / row / wave reductions built on them
template <int C>
__device__ __forceinline__ double dppd(double v) {
    const unsigned long long b = __builtin_bit_cast(unsigned long long, v);
    const unsigned lo = (unsigned)__builtin_amdgcn_update_dpp(0, (int)(unsigned)b, C, 0xF, 0xF, false);
    const unsigned hi = (unsigned)__builtin_amdgcn_update_dpp(0, (int)(unsigned)(b >> 32), C, 0xF, 0xF, false);
    return __builtin_bit_cast(double, ((unsigned long long)hi << 32) | lo);
}
__device__ __forceinline__ double rdld(double v, int l) {
    const unsigned long long b = __builtin_bit_cast(unsigned long long, v);
    const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)b, l);
    const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)(b >> 32), l);
    return __builtin_bit_cast(double, ((unsigned long long)hi << 32) | lo);
}
__device__ __forceinline__ double qsumd(double v) {   // over the 4 lanes of a quad, every lane
    v += dppd<0xB1>(v);
    return v + dppd<0x4E>(v);
}
__device__ __forceinline__ double wsumd(double v) {   // over the wave, uniform (fixed order)
    v = qsumd(v);
    v += dppd<0x141>(v);
    v += dppd<0x140>(v);
    return (rdld(v, 0) + rdld(v, 16)) + (rdld(v, 32) + rdld(v, 48));
}
__device__ __forceinline__ double wmaxd(double v) {
    v = fmax(v, dppd<0xB1>(v));
    v = fmax(v, dppd<0x4E>(v));
    v = fmax(v, dppd<0x141>(v));
    v = fmax(v, dppd<0x140>(v));
    return fmax(fmax(rdld(v, 0), rdld(v, 16)), fmax(rdld(v, 32), rdld(v, 48)));
}
template <int C>
__device__ __forceinline__ int dppi(int v) { return __builtin_amdgcn_update_dpp(0, v, C, 0xF, 0xF, false); }
// ordering of LDS traffic between the lanes of one wave (phases run by a single wave)
__device__ __forceinline__ void wsync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// ---------------------------------------------------------------------------------------
// R = X X^H / K on the f64 matrix cores (MUSIC_1D.m:28 in double).  Same decomposition as
// k_music_cov: one workgroup per instance, split-K over the 4 waves, lane l loads channels
// 4(l&15)..+3 of snapshot 4s + (l>>4) (64 B), and that register is both the A and the B operand
// of v_mfma_f64_16x16x4_f64 (A[r][kk] = x_I, B[kk][r] = x_J; tile (I, J) holds R[4r+I][4s+J]).
// Re R = Xr Xr^T + Xi Xi^T is symmetric: its 10 upper tiles, 2 MFMAs each per step.  Im R =
// P - P^T with P = Xi Xr^T: P's 16 tiles, 1 MFMA each, and the antisymmetric part is formed once
// in the epilogue -- 36 MFMAs per step instead of 40 (Im R tile by tile as Xi_I Xr_J^T - Xr_I
// Xi_J^T).  The f64 C/D layout puts row (l>>4) + 4i, column l&15 in accumulator element i.
// ---------------------------------------------------------------------------------------
__global__ __launch_bounds__(MU_THREADS, 2) void k_music_cov64(int N, int K, const double2* __restrict__ X,
                                                              double2* __restrict__ R) {
    __shared__ double red[10 + 16][256];   // Re R upper tiles, then P's tiles; D[row][col] row-major
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int r = lane & 15, kk = lane >> 4;
    const double2* __restrict__ Xi = X + (size_t)blockIdx.x * K * N;
    f64x4 ar[10], ap[16];
#pragma unroll
    for (int t = 0; t < 10; ++t) ar[t] = f64x4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int t = 0; t < 16; ++t) ap[t] = f64x4{0.0, 0.0, 0.0, 0.0};
    const int nsteps = (K + 3) >> 2;
    // the snapshots as one buffer resource: an element past the instance (k >= K or channel >= N)
    // gets an out-of-range offset and reads 0, so the loads carry no branch -- a branch around
    // each load made the compiler wait (vmcnt(0)) for it on the spot, and the loads issued two
    // steps ahead did not overlap the MFMAs of the step between
    const __amdgpu_buffer_rsrc_t xrs =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<double2*>(Xi), (short)0, (int)((unsigned)K * (unsigned)N * 16u), 0x00020000);
    auto load = [&](int s, double (&xr)[4], double (&xi)[4]) {
        const int k = 4 * s + kk, c0 = 4 * r;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            // bit 31 set (past num_records) when k >= K or the channel >= N: arithmetic, not a
            // select, which the compiler turned into a branch per load
            const unsigned bad = ((unsigned)(K - 1 - k) | (unsigned)(N - 1 - c0 - i)) & 0x80000000u;
            const unsigned off = (((unsigned)k * (unsigned)N + (unsigned)(c0 + i)) * 16u) | bad;
            const double2 x = __builtin_bit_cast(double2, __builtin_amdgcn_raw_buffer_load_b128(xrs, (int)off, 0, 0));
            xr[i] = x.x;
            xi[i] = x.y;
        }
    };
    auto step = [&](const double (&xr)[4], const double (&xi)[4]) {
        int t = 0;
#pragma unroll
        for (int I = 0; I < 4; ++I)
#pragma unroll
            for (int J = I; J < 4; ++J, ++t) {
                ar[t] = __builtin_amdgcn_mfma_f64_16x16x4f64(xr[I], xr[J], ar[t], 0, 0, 0);
                ar[t] = __builtin_amdgcn_mfma_f64_16x16x4f64(xi[I], xi[J], ar[t], 0, 0, 0);
            }
#pragma unroll
        for (int I = 0; I < 4; ++I)
#pragma unroll
            for (int J = 0; J < 4; ++J) ap[4 * I + J] = __builtin_amdgcn_mfma_f64_16x16x4f64(xi[I], xr[J], ap[4 * I + J], 0, 0, 0);
    };
    double xr0[4], xi0[4], xr1[4], xi1[4];
    // steps s and s + 4 per iteration, each one's loads issued two steps ahead; a step past the
    // snapshots reads zeros (out-of-range offsets) and adds exact zeros, so the loop has no
    // data-dependent branch around a load
    load(w, xr0, xi0);
    load(w + 4, xr1, xi1);
    for (int s = w; s < nsteps; s += 8) {
        step(xr0, xi0);
        load(s + 8, xr0, xi0);
        step(xr1, xi1);
        load(s + 12, xr1, xi1);
    }
    for (int ww = 0; ww < 4; ++ww) {   // ordered cross-wave sum (deterministic)
        if (w == ww) {
#pragma unroll
            for (int v = 0; v < 4; ++v) {
                const int e = (kk + 4 * v) * 16 + r;   // D row (l>>4) + 4v, column l&15
#pragma unroll
                for (int t = 0; t < 10; ++t) red[t][e] = ww == 0 ? ar[t][v] : red[t][e] + ar[t][v];
#pragma unroll
                for (int t = 0; t < 16; ++t) red[10 + t][e] = ww == 0 ? ap[t][v] : red[10 + t][e] + ap[t][v];
            }
        }
        __syncthreads();
    }
    double2* __restrict__ Ri = R + (size_t)blockIdx.x * MU_NMAX * MU_NMAX;   // column-major, ld 64
    int t = 0;
    for (int I = 0; I < 4; ++I)
        for (int J = I; J < 4; ++J, ++t) {
            const int i = tid >> 4, j = tid & 15;
            const int a = 4 * i + I, b = 4 * j + J;
            // Im R[a][b] = P[a][b] - P[b][a]: P tile (I, J) element (i, j) and tile (J, I) element (j, i)
            const double pim = red[10 + 4 * I + J][tid] - red[10 + 4 * J + I][j * 16 + i];
            const double re = red[t][tid] / K, im = pim / K;   // X1*X1'/K: a division, as MATLAB
            if (a < N && b < N) {
                Ri[a + MU_NMAX * b] = make_double2(re, im);
                if (I != J) Ri[b + MU_NMAX * a] = make_double2(re, -im);
            }
        }
}

// ---------------------------------------------------------------------------------------
// eig + MUSIC spectrum + findpeaks in double (MUSIC_1D.m:29-48): ONE 256-THREAD WORKGROUP PER
// INSTANCE, the matrix in registers.  Lane t holds column i = t >> 2, rows 16 (t & 3) .. +15
// (16 complex doubles): a quad of lanes is a column, so a column's sums are two DPP steps and
// the only LDS traffic of the reduction is the broadcast of v and w (and two partial sums).
//  1. Householder reduction to a real tridiagonal T (LAPACK zhetd2, lower): column k's quad
//     forms v_k (zlarfg) and keeps it; p = tau A v (lane = column, A Hermitian), w = p - tau/2
//     (p^H v) v, A -= v w^H + w v^H -- three barriers per step.
//  2. All eigenvalues of T by multisection, quad i -> the i-th smallest: the 4 lanes evaluate
//     the Sturm count (the leading minors' sign changes, division-free) at 4 interior points, 23 rounds
//     shrink the Gershgorin interval by 5^23 > 2^53 (to the rounding of the eigenvalue).
//  3. The M signal eigenvectors of T by inverse iteration (dlagtf / dlagts, lane j = vector j,
//     3 solves with modified Gram-Schmidt) in wave 0, then q_j = H_0 ... H_{n-2} y_j, the
//     reflectors applied by their own quads.
//  4. den(s) = |a(s) - Q_s Q_s^H a(s)|^2 = sum_j |Q_n^H a(s)|^2 (MUSIC_1D.m:37), lane = angle.
//  5. P = 1 ./ den, P_dB = 10 log10(P / max P), findpeaks + the M largest (MUSIC_1D.m:37-47).
// ---------------------------------------------------------------------------------------
#define ME_THREADS 256
#define ME_SECT 23     // multisection rounds with 4 interior points: 5^23 > 2^53
#define ME_PW_MIN 3    // block power iterations of the fast path (each with A^2) before the first
#define ME_PW_MAX 8    // convergence test, and at most (then the full path)


#define ME_SECT65 9    // rounds with 64 interior points: 65^9 > 2^53
// Floor of the squared off-diagonal entries the Sturm count reads (e2[], not ee[]): an exactly
// zero minor p_r must act as dstebz's q_r = -pivmin, i.e. a sign change after which
// p_{r+1} = -e_r^2 p_{r-1} carries on with the opposite sign.  With e_r^2 = 0 (a decoupled row or
// the pad rows) p_{r+1} would be 0 again and flip once more; at e_r^2 >= 2^-600 it is not.  The
// count runs on T scaled by 2^-s, 2^s ~ ||T|| (exact: a power of two), so the floor is relative --
// the eigenvalues move by at most ~2^-300 ||T|| and the solver is scale-invariant like eig.
#define ME_E2MIN 0x1p-600
#ifndef ME_WPS
#define ME_WPS 4     // waves per SIMD the register budget is sized for (4 instances per CU)
#endif
#define ME_VW 68                         // padded length of a v / w buffer
#define ME_PX(j) ((j) + ((j) >> 4))      // row j's slot in it
// the inverse iteration's [5][64][M] LU / y array; the back-transform stages a wave's 16
// reflectors ([16][ME_VW] complex) in the same space once the vectors have left it
__host__ __device__ constexpr int me_lu_doubles(int M) { return 5 * 64 * M > 32 * ME_VW ? 5 * 64 * M : 32 * ME_VW; }
__host__ __device__ constexpr size_t me_lds_bytes(int M, int S) {
    return (size_t)4 * ME_VW * 16 + 64 * 16 + 8 * 16 + 3 * 68 * 8 + 64 * 8 + (size_t)me_lu_doubles(M) * 8 + (size_t)M * 64 * 16 +
           ((size_t)S + 8) * 8 + 8 * 16;
}

// ---- Fast path of a peaks-only call (the caller reads no eigenvalues, M <= 4): the signal
// subspace span{q_1..q_M} of R -- all that den(s) = |a - Q_s Q_s^H a|^2 needs (MUSIC_1D.m:31-37)
// -- by orthogonal (block power) iteration instead of the full tridiagonal eigensolver: steps
// X <- orth(A^2 X) (CholeskyQR applied twice), M columns, tested for convergence after each step
// from the ME_PW_MIN-th to the ME_PW_MAX-th.  Accepted only with a proof that
// span(X) is within 1e-12 (sin of the largest principal angle) of the M leading eigenvectors:
// with H = X^H A X, E = A X - X H and C the compression of A to span(X)'s complement,
// ||A||_F^2 = ||H||_F^2 + 2 ||E||_F^2 + ||C||_F^2, so every eigenvalue of A outside the leading
// M is <= ||C||_F + ||E||_F (Weyl) =: c; if H - mu I is positive definite for mu = c + (1 + 1e12)
// ||E||_F (a Cholesky test), the gap between span(X)'s Ritz values and the rest exceeds 1e12
// ||E||_F, and Davis-Kahan bounds the angle by ||E||_F / gap <= 1e-12.  Otherwise (a small gap:
// slow convergence, or a matrix too degenerate for CholeskyQR) the caller runs the full path.  A
// is scaled by a power of two (exact) so that the iteration's magnitudes stay near 1 at any
// scale.  Uniform over the workgroup; lane t holds column i = t >> 2, rows 16 q .. +15 (q = t & 3).
// Packed S x S Hermitian matrices (pidx): the diagonal (reals) then the upper triangle (re, im).
template <int S>
__host__ __device__ constexpr int pidx_d(int c) { return c; }
template <int S>
__host__ __device__ constexpr int pidx_o(int c, int d) {   // c < d: re at the index, im at + 1
    int k = S;
    for (int cc = 0; cc < S; ++cc)
        for (int dd = cc + 1; dd < S; ++dd) {
            if (cc == c && dd == d) return k;
            k += 2;
        }
    return k;
}
// Cholesky of a packed S x S Hermitian matrix (in place: L's diagonal, L[d][c] for c < d stored at
// pidx_o(c, d) as L[d][c]); false unless positive definite
template <int S>
__device__ __forceinline__ bool me_chol_p(double (&G)[S * S]) {
    bool ok = true;
#pragma unroll
    for (int c = 0; c < S; ++c) {
        double d = G[pidx_d<S>(c)];
#pragma unroll
        for (int k = 0; k < c; ++k) {
            const int o = pidx_o<S>(k, c);   // L[c][k]
            d -= G[o] * G[o] + G[o + 1] * G[o + 1];
        }
        ok = ok && d > 0.0 && d < 1e300;
        const double lcc = sqrt(fmax(d, 1e-300)), il = 1.0 / lcc;
        G[pidx_d<S>(c)] = lcc;
#pragma unroll
        for (int r = c + 1; r < S; ++r) {   // L[r][c] = (G[r][c] - sum_k L[r][k] conj(L[c][k])) / L[c][c]
            const int o = pidx_o<S>(c, r);  // holds conj-pair G[c][r] = conj(G[r][c]) on entry
            double xr = G[o], xi = -G[o + 1];
#pragma unroll
            for (int k = 0; k < c; ++k) {
                const int orr = pidx_o<S>(k, r), oc = pidx_o<S>(k, c);   // L[r][k], L[c][k]
                xr -= G[orr] * G[oc] + G[orr + 1] * G[oc + 1];
                xi -= G[orr + 1] * G[oc] - G[orr] * G[oc + 1];
            }
            G[o] = xr * il;
            G[o + 1] = xi * il;
        }
    }
    return ok;
}
// y <- y L^{-H} for the row vector y (z L^H = y; L packed as me_chol_p leaves it)
template <int S>
__device__ __forceinline__ void me_trsm_p(double2 (&y)[S], const double (&L)[S * S]) {
#pragma unroll
    for (int d = 0; d < S; ++d) {
        double2 v = y[d];
#pragma unroll
        for (int c = 0; c < d; ++c) {   // (L^H)[c][d] = conj(L[d][c])
            const int o = pidx_o<S>(c, d);
            v = zsub(v, zm(y[c], make_double2(L[o], -L[o + 1])));
        }
        y[d] = zsc(1.0 / L[pidx_d<S>(d)], v);
    }
}

template <int M>
__device__ bool me_fast_subspace(const double2 (&a)[16], int n, int t, int lane, int w, int i, int q,
                                 double2* __restrict__ Qb, double2* __restrict__ Yb, double* __restrict__ gp,
                                 double2* __restrict__ Qs) {
    constexpr int S = M;
    constexpr int NV = S * S;
    const double2 z2 = make_double2(0.0, 0.0);
    int gb = 0;   // the reduction scratch alternates between two halves (one barrier per sum)
    // sum over the 64 rows (each quad's lane q == 0, or every lane: all) and the 4 waves
    auto reduce = [&](double (&v)[NV], bool all) {
#pragma unroll
        for (int k = 0; k < NV; ++k) v[k] = wsumd(all || q == 0 ? v[k] : 0.0);
        double* g = gp + gb * 4 * NV;
        if (lane == 0)
#pragma unroll
            for (int k = 0; k < NV; ++k) g[w * NV + k] = v[k];
        __syncthreads();
#pragma unroll
        for (int k = 0; k < NV; ++k) v[k] = (g[k] + g[NV + k]) + (g[2 * NV + k] + g[3 * NV + k]);
        gb ^= 1;
    };
    // packed X^H Y over the rows (x, y: this quad's row of X and Y)
    auto herm = [&](const double2 (&x)[S], const double2 (&y)[S], double (&G)[NV]) {
#pragma unroll
        for (int c = 0; c < S; ++c) {
            G[pidx_d<S>(c)] = zmc(x[c], y[c]).x;
#pragma unroll
            for (int d = c + 1; d < S; ++d) {
                const double2 e = zmc(x[c], y[d]);
                G[pidx_o<S>(c, d)] = e.x;
                G[pidx_o<S>(c, d) + 1] = e.y;
            }
        }
        reduce(G, false);
    };
    // the scale 2^-e with max |a_ij| in [1/2, 1) after it (a power of two: exact), and ||sA A||_F^2
    double am = 0.0, a2 = 0.0;
#pragma unroll
    for (int u = 0; u < 16; ++u) am = fmax(am, fmax(fabs(a[u].x), fabs(a[u].y)));
    am = wmaxd(am);
    if (lane == 0) gp[8 * NV + w] = am;
    __syncthreads();
    am = fmax(fmax(gp[8 * NV + 0], gp[8 * NV + 1]), fmax(gp[8 * NV + 2], gp[8 * NV + 3]));
    if (!(am > 0.0) || !(am < 1e300)) return false;   // uniform
    const double sA = __builtin_amdgcn_ldexp(1.0, -__builtin_amdgcn_frexp_exp(am));
    {
        double v[NV];
#pragma unroll
        for (int k = 0; k < NV; ++k) v[k] = 0.0;
        // squares of the scaled entries (|sA a| in [0, 1)): summed unscaled, entries below ~1e-154
        // would underflow and leave ||C|| assumed 0 in the bound below
#pragma unroll
        for (int u = 0; u < 16; ++u) {
            const double xr = a[u].x * sA, xi = a[u].y * sA;
            a2 = fma(xr, xr, fma(xi, xi, a2));
        }
        v[0] = a2;
        reduce(v, true);
        a2 = v[0];
    }
    // y = sA A X (A Hermitian: row i of A X = sum_j conj(A(j, i)) X[j], quad i's column)
    auto matvec = [&](const double2* X, double2 (&y)[S]) {
#pragma unroll
        for (int c = 0; c < S; ++c) {
            double px4[4] = {0.0, 0.0, 0.0, 0.0}, py4[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
            for (int u = 0; u < 16; ++u) {
                const double2 xj = X[c * ME_VW + ME_PX(16 * q + u)];
                px4[u & 3] = fma(a[u].x, xj.x, fma(a[u].y, xj.y, px4[u & 3]));
                py4[u & 3] = fma(a[u].x, xj.y, fma(-a[u].y, xj.x, py4[u & 3]));
            }
            const double px = qsumd((px4[0] + px4[1]) + (px4[2] + px4[3]));
            const double py = qsumd((py4[0] + py4[1]) + (py4[2] + py4[3]));
            y[c] = make_double2(px * sA, py * sA);
            __builtin_amdgcn_sched_barrier(0);   // one column's 16 LDS loads in flight at a time (128 VGPRs)
        }
    };
    // start: fixed unit-modulus vectors (deterministic; not orthogonal to an eigenvector in practice)
    for (int e = t; e < S * 64; e += ME_THREADS) {
        const int c = e >> 6, j = e & 63;
        double sn, cs;
        sincos(0.7 * (double)(j * (2 * c + 1)) + 1.3 * (double)c, &sn, &cs);
        Qb[c * ME_VW + ME_PX(j)] = j < n ? make_double2(cs, sn) : z2;
    }
    __syncthreads();
    bool ok = true, conv = false;
    double2 x[S];
    for (int it = 0; it < ME_PW_MAX && ok && !conv; ++it) {   // uniform
        {
            double2 y[S], z[S];
            matvec(Qb, y);
            if (q == 0)
#pragma unroll
                for (int c = 0; c < S; ++c) Yb[c * ME_VW + ME_PX(i)] = y[c];
            __syncthreads();
            matvec(Yb, z);   // sA^2 A^2 X
#pragma unroll
            for (int pass = 0; pass < 2; ++pass) {   // CholeskyQR2: orthonormal to rounding
                double G[NV];
                herm(z, z, G);
                ok = me_chol_p<S>(G) && ok;
                me_trsm_p<S>(z, G);
            }
            if (q == 0)
#pragma unroll
                for (int c = 0; c < S; ++c) Qb[c * ME_VW + ME_PX(i)] = z[c];
            __syncthreads();
#pragma unroll
            for (int c = 0; c < S; ++c) x[c] = z[c];
        }
        if (!ok || it + 1 < ME_PW_MIN) continue;
        // the proof of convergence (see above): H = X^H A X, E = A X - X H, c bounds the rest
        double2 y[S];
        matvec(Qb, y);
        double H[NV];
        herm(x, y, H);
        double h2 = 0.0, e2 = 0.0;
#pragma unroll
        for (int c = 0; c < S; ++c) {
            h2 += H[pidx_d<S>(c)] * H[pidx_d<S>(c)];
#pragma unroll
            for (int d = c + 1; d < S; ++d)
                h2 += 2.0 * (H[pidx_o<S>(c, d)] * H[pidx_o<S>(c, d)] + H[pidx_o<S>(c, d) + 1] * H[pidx_o<S>(c, d) + 1]);
        }
#pragma unroll
        for (int j = 0; j < S; ++j) {   // row i of E, column j
            double2 e = y[j];
#pragma unroll
            for (int k = 0; k < S; ++k) {
                const double2 hkj = k == j ? make_double2(H[pidx_d<S>(k)], 0.0)
                                           : (k < j ? make_double2(H[pidx_o<S>(k, j)], H[pidx_o<S>(k, j) + 1])
                                                    : make_double2(H[pidx_o<S>(j, k)], -H[pidx_o<S>(j, k) + 1]));
                e = zsub(e, zm(x[k], hkj));
            }
            e2 += e.x * e.x + e.y * e.y;
        }
        {
            double v[NV];
#pragma unroll
            for (int k = 0; k < NV; ++k) v[k] = 0.0;
            v[0] = e2;
            reduce(v, false);
            e2 = v[0];
        }
        // (1e-14 a2: the rounding of the difference, so that cb stays an upper bound)
        const double en = sqrt(e2), cb = sqrt(fmax(a2 - h2 - 2.0 * e2, 0.0) + 1e-14 * a2);
        const double mu = cb + en * (1.0 + 1e12);
#pragma unroll
        for (int c = 0; c < S; ++c) H[pidx_d<S>(c)] -= mu;
        conv = me_chol_p<S>(H);   // H - mu I positive definite: the proof holds (uniform)
    }
    if (!conv) return false;   // uniform
    if (q == 0)
#pragma unroll
        for (int j = 0; j < M; ++j) Qs[j * 64 + i] = x[j];
    __syncthreads();
    return true;
}

// FAST (peaks-only launches, neig <= 4): try me_fast_subspace first.  A separate instantiation, so
// that the launches that read every eigenvalue run the full path without the fast path's registers.
template <int M, bool FAST>
__global__ __launch_bounds__(ME_THREADS, ME_WPS) void k_music_eig64(int N, int S, int neig, double spec_tol,
                                                          const double2* __restrict__ R,
                                                          const double2* __restrict__ S1T, int Spad,
                                                          double* __restrict__ spec_db, double* __restrict__ eig_out,
                                                          int* __restrict__ peaks_out, unsigned long long* __restrict__ trace) {
    // trace (diagnostic builds, RSP_MUSIC_TRACE=1): s_memrealtime at the phase boundaries
#define ME_STAMP(ix) \
    if (trace && threadIdx.x == 0) trace[(size_t)blockIdx.x * 8 + (ix)] = wall_clock64()
    ME_STAMP(0);
    extern __shared__ __attribute__((aligned(16))) double2 lds64[];
    // v and w of a step, double-buffered by k parity, each row j at ME_PX(j) (a pad every 16: the
    // 4 row blocks a wave's quads read together, 16 q + u, fall on distinct banks instead of one)
    double2* vb = lds64;                 // [2][68] v
    double2* wb = vb + 2 * ME_VW;        // [2][68] w
    double2* taus = wb + 2 * ME_VW;      // [64]
    double2* red = taus + 64;            // [8] per-wave partial sums
    double* dd = reinterpret_cast<double*>(red + 8);   // T diagonal (+ 4 pad rows for the Sturm count)
    double* ee = dd + 68;                // T off-diagonal (beta_k, signed)
    double* e2 = ee + 68;                // beta_k^2 (+ pad)
    double* lam = e2 + 68;               // ascending eigenvalues
    double* lu = lam + 64;               // [5][64][M]: U diag, U super 1, U super 2, mult, y
    double2* Qs = reinterpret_cast<double2*>(lu + me_lu_doubles(M));   // [M][64]
    double* den = reinterpret_cast<double*>(Qs + M * 64);        // [S]
    int* ired = reinterpret_cast<int*>(den + S + 8);             // [8] + the peak selection
    double* dred = den + S;                                      // [8]
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    const int i = t >> 2, q = t & 3;
    const int n = N;
    const double2 z2 = make_double2(0.0, 0.0);
    double2 a[16];   // A(16 q + u, i)
    {
        const double2* __restrict__ Ri = R + (size_t)blockIdx.x * MU_NMAX * MU_NMAX;
#pragma unroll
        for (int u = 0; u < 16; ++u) {
            const int j = 16 * q + u;
            a[u] = (i < n && j < n) ? Ri[j + MU_NMAX * i] : z2;
        }
    }
    // ---- 0. peaks-only calls: the signal subspace by block power iteration when it converges
    //         (me_fast_subspace); otherwise, and whenever every eigenvalue is requested, 1.-3.
    bool fast = false;
    if constexpr (FAST && M <= 4) {
        if (neig <= 4 && M + 1 <= n) {
            double2* Qb = reinterpret_cast<double2*>(lu);
            fast = me_fast_subspace<M>(a, n, t, lane, w, i, q, Qb, Qb + (M + 1) * ME_VW,
                                       reinterpret_cast<double*>(Qb + 2 * (M + 1) * ME_VW), Qs);
        }
    }
    // ---- 4. den(s) = |a(s) - Q_s (Q_s^H a(s))|^2, lane = angle; returns max_s 1 / den(s)
    auto den_pmax = [&]() -> double {
        for (int s = t; s < S; s += ME_THREADS) {
            double2 cf[M];
#pragma unroll
            for (int m = 0; m < M; ++m) cf[m] = z2;
            for (int c = 0; c < n; ++c) {
                const double2 av = S1T[(size_t)c * Spad + s];
#pragma unroll
                for (int m = 0; m < M; ++m) cf[m] = zadd(cf[m], zmc(Qs[m * 64 + c], av));
            }
            double r2 = 0.0;
            for (int c = 0; c < n; ++c) {
                double2 rr = S1T[(size_t)c * Spad + s];
#pragma unroll
                for (int m = 0; m < M; ++m) rr = zsub(rr, zm(Qs[m * 64 + c], cf[m]));
                r2 += rr.x * rr.x + rr.y * rr.y;
            }
            den[s] = r2;
        }
        __syncthreads();
        double pm = 0.0;
        for (int s = t; s < S; s += ME_THREADS) pm = fmax(pm, 1.0 / den[s]);
        pm = wmaxd(pm);
        if (lane == 0) dred[w] = pm;
        __syncthreads();
        const double r = fmax(fmax(dred[0], dred[1]), fmax(dred[2], dred[3]));
        __syncthreads();   // dred is reused
        return r;
    };
    double pmax = 0.0;
    bool have_den = false;
    if constexpr (FAST) {
        // A call that reads the spectrum (spec_tol > 0) keeps the fast subspace only if it also
        // bounds the spectrum: sin(angle) <= 1e-12 to the signal eigenvectors moves the projector
        // by <= 1e-12, so each den(s) by <= e0 = 1e-12 |a(s)|^2 = 1e-12 n (unit-modulus steering),
        // and P_dB(s) = 10 log10(den_min / den(s)) by <= (20 / ln 10) e / (1 - e), e = e0 / den_min
        // = e0 pmax.  Otherwise the full eigensolver (uniform).
        if (fast && spec_tol > 0.0) {
            pmax = den_pmax();
            have_den = true;
            const double e = 1e-12 * n * pmax;
            if (!(e < 0.5 && 8.6858896380650366 * e / (1.0 - e) <= spec_tol)) fast = have_den = false;
        }
    }
    if (!fast) {
    // ---- 1. tridiagonalisation
    for (int k = 0; k < n - 1; ++k) {
        double2* vk = vb + ME_VW * (k & 1);
        double2* wk = wb + ME_VW * (k & 1);
        if (w == (k >> 4)) {   // the wave holding column k (uniform)
            // column k through LDS (wk of this step is free until its w is written): lane = row
            double2* cb = wk;
            if (i == k) {
#pragma unroll
                for (int u = 0; u < 16; ++u) cb[ME_PX(16 * q + u)] = a[u];
            }
            wsync();
            const double2 c = cb[ME_PX(lane)];
            const double xn = wsumd(lane >= k + 2 ? c.x * c.x + c.y * c.y : 0.0);   // rows >= n are 0
            const double2 al = make_double2(rdld(c.x, k + 1), rdld(c.y, k + 1));
            const double dk = rdld(c.x, k);
            double2 tau = z2, scale = z2;
            double beta = al.x;
            if (xn > 0.0 || al.y != 0.0) {   // zlarfg
                beta = -copysign(sqrt(al.x * al.x + al.y * al.y + xn), al.x);
                tau = make_double2((beta - al.x) / beta, -al.y / beta);
                const double2 dn = make_double2(al.x - beta, al.y);
                const double qd = 1.0 / (dn.x * dn.x + dn.y * dn.y);
                scale = make_double2(dn.x * qd, -dn.y * qd);
            }
            vk[ME_PX(lane)] = lane == k + 1 ? make_double2(1.0, 0.0) : (lane >= k + 2 ? zm(c, scale) : z2);
            if (lane == 0) {
                taus[k] = tau;
                dd[k] = dk;
                ee[k] = beta;   // e2 (scaled, floored) is formed in phase 2
            }
        }
        __syncthreads();
        if (w == (k >> 4) && i == k) {   // column k keeps v_k for the back-transformation
#pragma unroll
            for (int u = 0; u < 16; ++u) a[u] = vk[ME_PX(16 * q + u)];
        }
        const double2 tau = taus[k];
        if (tau.x == 0.0 && tau.y == 0.0) continue;   // H_k = I (uniform)
        // columns <= k are finished: their quads (whole waves, late in the reduction) skip the work
        const bool act = i > k && i < n;
        double2 p = z2;
        if (act) {   // uniform per quad
            // sum_j conj(A(j,i)) v_j in 4 interleaved partial sums (dependent chains of 8 FMAs
            // instead of 32)
            double px4[4] = {0.0, 0.0, 0.0, 0.0}, py4[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
            for (int u = 0; u < 16; ++u) {
                const double2 vj = vk[ME_PX(16 * q + u)];
                px4[u & 3] = fma(a[u].x, vj.x, fma(a[u].y, vj.y, px4[u & 3]));
                py4[u & 3] = fma(a[u].x, vj.y, fma(-a[u].y, vj.x, py4[u & 3]));
            }
            double px = (px4[0] + px4[1]) + (px4[2] + px4[3]);
            double py = (py4[0] + py4[1]) + (py4[2] + py4[3]);
            px = qsumd(px);
            py = qsumd(py);
            p = zm(tau, make_double2(px, py));
        }
        const double2 vi = vk[ME_PX(i)];
        double2 pv = q == 0 ? zmc(p, vi) : z2;                                  // p^H v
        pv.x = wsumd(pv.x);
        pv.y = wsumd(pv.y);
        if (lane == 0) red[w] = pv;
        __syncthreads();
        const double2 sp = zadd(zadd(red[0], red[1]), zadd(red[2], red[3]));
        const double2 alpha = zsc(-0.5, zm(tau, sp));
        const double2 wi = act ? zadd(p, zm(alpha, vi)) : z2;
        if (q == 0) wk[ME_PX(i)] = wi;
        __syncthreads();
        if (act) {   // A(j, i) -= v_j conj(w_i) + w_j conj(v_i) (v_j = w_j = 0 for j <= k): 8 FMAs
#pragma unroll
            for (int u = 0; u < 16; ++u) {
                const int j = 16 * q + u;
                const double2 vj = vk[ME_PX(j)], wj = wk[ME_PX(j)];
                double ax = a[u].x, ay = a[u].y;
                ax = fma(-vj.x, wi.x, ax);
                ax = fma(-vj.y, wi.y, ax);
                ax = fma(-wj.x, vi.x, ax);
                ax = fma(-wj.y, vi.y, ax);
                ay = fma(-vj.y, wi.x, ay);
                ay = fma(vj.x, wi.y, ay);
                ay = fma(-wj.y, vi.x, ay);
                ay = fma(wj.x, vi.y, ay);
                a[u] = make_double2(ax, ay);
            }
        }
    }
    if (w == ((n - 1) >> 4)) {
        double dl = 0.0;
#pragma unroll
        for (int u = 0; u < 16; ++u)
            if (u == ((n - 1) & 15) && i == n - 1 && q == ((n - 1) >> 4)) dl = a[u].x;   // u vs a uniform: no per-lane row index
        dl = qsumd(dl);
        if (i == n - 1 && q == 0) dd[n - 1] = dl;
    }
    __syncthreads();
    ME_STAMP(1);
    // ---- 2. eigenvalues by multisection (quad i -> the i-th smallest)
    {
        double glo = 1.0e300, ghi = -1.0e300, emax = 0.0;
        for (int r = 0; r < n; ++r) {   // Gershgorin
            const double rad = (r > 0 ? fabs(ee[r - 1]) : 0.0) + (r < n - 1 ? fabs(ee[r]) : 0.0);
            glo = fmin(glo, dd[r] - rad);
            ghi = fmax(ghi, dd[r] + rad);
            if (r < n - 1) emax = fmax(emax, ee[r] * ee[r]);
        }
        const double tn = fmax(fabs(glo), fabs(ghi));
        const double pivmin = 2.2250738585072014e-308 * fmax(1.0, emax);   // dstebz PIVMIN
        double lo = glo - 4.4e-16 * tn - 2.0 * pivmin, hi = ghi + 4.4e-16 * tn + 2.0 * pivmin;
        // # eigenvalues of T below x: sign changes of the leading minors p_r = det(T_r - x I),
        // p_r = (d_r - x) p_{r-1} - e_{r-1}^2 p_{r-2} -- the division-free form of dstebz's
        // q_r = p_r / p_{r-1} (its dependent chain is one FMA per row instead of a reciprocal).
        // A zero minor counts as a sign change, as q_r = 0 -> -pivmin does there; both minors
        // are rescaled by a power of two every 4 rows (no overflow or underflow).
        // rows n .. n + 3 pad the count to whole blocks of 4: d = ghi + 1 > every x of the
        // search and e^2 = ME_E2MIN keep the minors' signs (p_r ~ (d - x) p_{r-1}, d - x > 0)
        // The count runs on 2^-s T, 2^s ~ ||T|| (x, d scaled as they are read; e^2 formed here from
        // the scaled e): powers of two, so for any T whose scaled entries neither underflow nor
        // overflow the signs are those of T itself, and the floor ME_E2MIN is relative to ||T||.
        const double isg = __builtin_amdgcn_ldexp(1.0, -__builtin_amdgcn_frexp_exp(tn));
        __syncthreads();   // every lane has read dd / ee (Gershgorin) before the pad rows land
        for (int r = t; r < n - 1; r += ME_THREADS) {
            const double es = ee[r] * isg;
            e2[r] = fmax(es * es, ME_E2MIN);
        }
        if (t < 4) {
            dd[n + t] = ghi + fmax(tn, 1.0);   // > hi at any scale
            e2[n - 1 + t] = ME_E2MIN;
        }
        __syncthreads();
        auto sturm = [&](double xu) -> int {
            const double x = xu * isg;
            double pm = 1.0, pc = dd[0] * isg - x;
            bool sc = !(pc > 0.0);   // effective sign of p_0 (zero -> negative, as -pivmin)
            int c = sc;
            double dn = dd[1] * isg, en = e2[0];   // row r's (d_r, e_{r-1}^2), loaded a row ahead
            for (int r0 = 1; r0 < n; r0 += 4) {
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const int r = r0 + j;
                    const double d = dn, e = en;
                    dn = dd[r + 1] * isg;   // r + 1 <= n + 3 (padded)
                    en = e2[r];
                    const double pn = fma(d - x, pc, -e * pm);
                    const bool sn = (pn < 0.0) | ((pn == 0.0) & !sc);
                    c += sn ^ sc;
                    sc = sn;
                    pm = pc;
                    pc = pn;
                }
                const int ex = __builtin_amdgcn_frexp_exp(pc);   // rescale both by 2^-ex
                pc = __builtin_amdgcn_ldexp(pc, -ex);
                pm = __builtin_amdgcn_ldexp(pm, -ex);
            }
            return c;
        };
        if (neig <= 4) {
            // Only the neig <= 4 largest (the M signal eigenvalues, when the caller does not read
            // them all): one wave per eigenvalue, its 64 lanes at the 64 interior points of the
            // interval (65-section), 9 rounds (65^9 > 2^53) of one Sturm chain each instead of 23.
            // Lane l's count c_l is non-decreasing in l, so the lanes with c_l <= ie are a prefix
            // of m lanes and the ie-th smallest eigenvalue lies in [x_{m-1}, x_m].
            const int ie = n - 1 - w;   // ascending index of wave w's eigenvalue
            if (w < neig) {
                for (int it = 0; it < ME_SECT65; ++it) {
                    const double h = (hi - lo) * (1.0 / 65.0);
                    const int c = sturm(lo + h * (lane + 1));
                    const int m = __builtin_popcountll(__builtin_amdgcn_ballot_w64(c <= ie));
                    const double nl = m == 0 ? lo : lo + h * m;
                    const double nh = m == 64 ? hi : lo + h * (m + 1);
                    lo = nl;
                    hi = nh;
                }
                if (lane == 0) {
                    const double l = 0.5 * (lo + hi);
                    lam[ie] = l;
                    eig_out[(size_t)blockIdx.x * N + w] = l;   // descending (MUSIC_1D.m:31)
                }
            }
        } else if (i < n) {   // every eigenvalue: quad i -> the i-th smallest
            for (int it = 0; it < ME_SECT; ++it) {
                const double h = (hi - lo) * 0.2;
                const int c = sturm(lo + h * (q + 1));
                const int m = (dppi<0x00>(c) <= i) + (dppi<0x55>(c) <= i) + (dppi<0xAA>(c) <= i) + (dppi<0xFF>(c) <= i);
                const double nl = m == 0 ? lo : lo + h * m;
                const double nh = m == 4 ? hi : lo + h * (m + 1);
                lo = nl;
                hi = nh;
            }
            if (q == 0) {
                const double l = 0.5 * (lo + hi);
                lam[i] = l;
                eig_out[(size_t)blockIdx.x * N + (n - 1 - i)] = l;   // descending (MUSIC_1D.m:31)
            }
        }
    }
    __syncthreads();
    ME_STAMP(2);
    // ---- 3. signal eigenvectors of T: inverse iteration in wave 0 (lane j = vector j, then
    //         lane = component)
    if (w == 0) {
        double tnorm = 0.0;
        for (int r = 0; r < n; ++r)
            tnorm = fmax(tnorm, fabs(dd[r]) + (r > 0 ? fabs(ee[r - 1]) : 0.0) + (r < n - 1 ? fabs(ee[r]) : 0.0));
        const double ptol = 2.2e-16 * tnorm + 1e-300;
#define LU(arr, r) lu[((arr) * 64 + (r)) * M + lane]
        unsigned long long swp = 0ull;
        if (lane < M) {   // dlagtf on T - lambda_j I
            const double lj = lam[n - 1 - lane];
            double ak = dd[0] - lj;
            double bk = n > 1 ? ee[0] : 0.0;
            for (int k0 = 0; k0 < n - 1; k0 += 4) {   // 4 rows of T per LDS round trip
                double ckv[4], anv[4], bnv[4];
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const int k = min(k0 + j, n - 2);
                    ckv[j] = ee[k];
                    anv[j] = dd[k + 1] - lj;
                    bnv[j] = k < n - 2 ? ee[k + 1] : 0.0;
                }
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const int k = k0 + j;
                    if (k < n - 1) {   // branch-free over the lanes' interchange choices, one division
                        const double ck = ckv[j], an = anv[j], bn = bnv[j];
                        const bool keep = fabs(ak) >= fabs(ck);
                        const double a0 = fabs(ak) < ptol ? copysign(ptol, ak) : ak;
                        const double r0 = 1.0 / (keep ? a0 : ck);
                        const double mult = (keep ? ck : ak) * r0;
                        LU(0, k) = r0;
                        LU(1, k) = keep ? bk : an;
                        LU(2, k) = keep ? 0.0 : bn;
                        LU(3, k) = mult;
                        if (!keep) swp |= 1ull << k;
                        const double akn = keep ? an - mult * bk : bk - mult * an;
                        bk = keep ? bn : -mult * bn;
                        ak = akn;
                    }
                }
            }
            LU(0, n - 1) = 1.0 / (fabs(ak) < ptol ? copysign(ptol, ak) : ak);   // U's diagonal stored inverted:
                                                                                   // the solves multiply
            for (int r = 0; r < n; ++r) LU(4, r) = 1.0 + 0.0625 * (double)((r * 37 + lane * 11) % 17);   // start
        }
        ME_STAMP(7);   // diagnostic builds: the end of dlagtf (printed apart)
        for (int it = 0; it < MU_ITER; ++it) {
            if (lane < M) {   // dlagts, 4 rows at a time: the rows' LDS loads issue ahead of the chain
                double yk = LU(4, 0);
                for (int k0 = 0; k0 < n - 1; k0 += 4) {
                    double ynv[4], mlv[4];
#pragma unroll
                    for (int j = 0; j < 4; ++j) {   // rows past n - 2 read row n - 2 again (unused)
                        const int k = min(k0 + j, n - 2);
                        ynv[j] = LU(4, k + 1);
                        mlv[j] = LU(3, k);
                    }
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        const int k = k0 + j;
                        if (k < n - 1) {
                            if (swp >> k & 1ull) {
                                LU(4, k) = ynv[j];
                                yk = yk - mlv[j] * ynv[j];
                            } else {
                                LU(4, k) = yk;
                                yk = ynv[j] - mlv[j] * yk;
                            }
                        }
                    }
                }
                double y1 = yk * LU(0, n - 1), y2 = 0.0;
                LU(4, n - 1) = y1;
                for (int k0 = n - 2; k0 >= 0; k0 -= 4) {
                    double r4[4], u1[4], u2[4], u0[4];
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        const int k = max(k0 - j, 0);
                        r4[j] = LU(4, k);
                        u1[j] = LU(1, k);
                        u2[j] = LU(2, k);
                        u0[j] = LU(0, k);
                    }
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        const int k = k0 - j;
                        if (k >= 0) {
                            const double yk2 = (r4[j] - u1[j] * y1 - u2[j] * y2) * u0[j];
                            LU(4, k) = yk2;
                            y2 = y1;
                            y1 = yk2;
                        }
                    }
                }
            }
            wsync();
            for (int j = 0; j < M; ++j) {   // modified Gram-Schmidt (lane = component)
                double yj = lane < n ? lu[(4 * 64 + lane) * M + j] : 0.0;
                for (int ii = 0; ii < j; ++ii) {
                    const double yi = lane < n ? lu[(4 * 64 + lane) * M + ii] : 0.0;
                    yj -= wsumd(yi * yj) * yi;
                }
                yj /= sqrt(wsumd(yj * yj));
                if (lane < n) lu[(4 * 64 + lane) * M + j] = yj;
                wsync();
            }
        }
#undef LU
        for (int j = 0; j < M; ++j) Qs[j * 64 + lane] = make_double2(lane < n ? lu[(4 * 64 + lane) * M + j] : 0.0, 0.0);
    }
    __syncthreads();
    ME_STAMP(3);
    // q_j = H_0 H_1 ... H_{n-2} y_j, k descending: the reflectors of wave wv's 16 columns are
    // applied by wave wv with lane = row and the M vectors in registers (a wave's turn starts and
    // ends with them in Qs); v_k passes from its quad to the wave through a 1 KB LDS buffer
    for (int wv = 3; wv >= 0; --wv) {
        if (w == wv && 16 * wv <= n - 2) {
            double2 y[M];
#pragma unroll
            for (int j = 0; j < M; ++j) y[j] = Qs[j * 64 + lane];
            // the wave's reflectors (its 16 columns, quad i holds v_i) into LDS at once, so the
            // loop below only reads them (lu is dead: the vectors are in Qs)
            double2* blk = reinterpret_cast<double2*>(lu);   // [16][ME_VW]
            const int klast = min(n - 2, 16 * wv + 15);
            if (i <= klast) {
#pragma unroll
                for (int u = 0; u < 16; ++u) blk[(i - 16 * wv) * ME_VW + ME_PX(16 * q + u)] = a[u];
            }
            wsync();
            for (int k = klast; k >= 16 * wv; --k) {
                const double2 vl = blk[(k - 16 * wv) * ME_VW + ME_PX(lane)], tau = taus[k];
#pragma unroll
                for (int j = 0; j < M; ++j) {
                    double2 d = zmc(vl, y[j]);   // v^H y
                    d.x = wsumd(d.x);
                    d.y = wsumd(d.y);
                    y[j] = zsub(y[j], zm(vl, zm(tau, d)));
                }
            }
#pragma unroll
            for (int j = 0; j < M; ++j) Qs[j * 64 + lane] = y[j];
        }
        __syncthreads();
    }
    }   // !fast
    ME_STAMP(4);
    if (!have_den) pmax = den_pmax();
    ME_STAMP(5);
    // ---- 5. P = 1 ./ den, P_dB = 10 log10(P / max P) (MUSIC_1D.m:37-41)
    double* __restrict__ out = spec_db + (size_t)blockIdx.x * S;
    for (int s = t; s < S; s += ME_THREADS) {
        const double db = 10.0 * log10((1.0 / den[s]) / pmax);
        den[s] = db;
        out[s] = db;
    }
    __syncthreads();
    // findpeaks (MUSIC_1D.m:43) + the M largest, ties to the lower index (MUSIC_1D.m:44-47)
    unsigned pkm = 0u;   // bit tt: s = t + 256 tt is a peak (S <= 4096)
    int npk = 0;
    for (int tt = 0; tt * ME_THREADS < S; ++tt) {
        const int s = t + ME_THREADS * tt;
        bool pk = false;
        if (s >= 1 && s < S - 1 && den[s] > den[s - 1]) {
            int u = s + 1;
            while (u < S && den[u] == den[s]) ++u;
            pk = u < S && den[u] < den[s];
        }
        if (pk) pkm |= 1u << tt;
        npk += pk;
    }
    npk = (int)wsumd((double)npk);
    if (lane == 0) ired[w] = npk;
    __syncthreads();
    int* po = peaks_out + (size_t)blockIdx.x * (MU_MMAX + 1);
    if (t == 0) {
        po[0] = (ired[0] + ired[1]) + (ired[2] + ired[3]);
    }
    __syncthreads();
    for (int rk = 0; rk < M; ++rk) {
        double bv = -1.0e300;
        int bs = 1 << 30;
        for (int tt = 0; tt * ME_THREADS < S; ++tt)
            if (pkm >> tt & 1u) {
                const int s = t + ME_THREADS * tt;
                if (den[s] > bv) { bv = den[s]; bs = s; }   // tt ascending: ties keep the lower s
            }
        const double gv = wmaxd(bv);
        int cand = bv == gv ? bs : (1 << 30);
        cand = min(cand, dppi<0xB1>(cand));
        cand = min(cand, dppi<0x4E>(cand));
        cand = min(cand, dppi<0x141>(cand));
        cand = min(cand, dppi<0x140>(cand));
        cand = min(min(__builtin_amdgcn_readlane(cand, 0), __builtin_amdgcn_readlane(cand, 16)),
                   min(__builtin_amdgcn_readlane(cand, 32), __builtin_amdgcn_readlane(cand, 48)));
        if (lane == 0) {
            dred[w] = gv;
            ired[w] = cand;
        }
        __syncthreads();
        double best = dred[0];
        for (int ww = 1; ww < 4; ++ww) best = fmax(best, dred[ww]);
        int gs = 1 << 30;
        for (int ww = 0; ww < 4; ++ww)
            if (dred[ww] == best) gs = min(gs, ired[ww]);
        if (gs < (1 << 30) && (gs % ME_THREADS) == t) pkm &= ~(1u << (gs / ME_THREADS));
        if (t == 0) po[1 + rk] = gs < (1 << 30) ? gs + 1 : 0;
        __syncthreads();
    }
    if (t == 0) {
        for (int rk = M; rk < MU_MMAX; ++rk) po[1 + rk] = 0;
        if (M < MU_MMAX) po[MU_MMAX] = fast ? 1 : 0;   // the slot past the M peaks: which path ran (rsp_music_fast_count)
    }
    ME_STAMP(6);
#undef ME_STAMP
}

}  // namespace

// =======================================================================================
// Host side: plan + C-ABI (include/rsp.h, MUSIC section)
// =======================================================================================
struct rsp_music_plan {
    int device = 0;
    int N = 0, K = 0, M = 0, S = 0, Spad = 0, max_batch = 0;
    bool f64 = true;              // RSP_C128 (MATLAB's complex double, default) or RSP_C64
    size_t xsz = 16;              // bytes of one snapshot sample
    double dl = 0.0;
    hipStream_t stream = nullptr;
    void* d_S1T = nullptr;        // steering table [64][Spad] (float2 / double2), zero rows for c >= N
    void* d_R = nullptr;          // [max_batch][64][64] complex
    void* d_X = nullptr;          // host-path staging [max_batch][K][N] (lazy)
    void* d_spec = nullptr;       // [max_batch][S] float / double
    void* d_eig = nullptr;        // [max_batch][N] float / double
    int* d_peaks = nullptr;       // [max_batch][MU_MMAX + 1]
    double2* d_src = nullptr;     // synthesis: source steering [MU_MMAX][N]
    double* d_amp = nullptr;      // [MU_MMAX]
    unsigned long long* d_trace = nullptr;   // RSP_MUSIC_TRACE: [max_batch][8] phase stamps (f32 eig)
    hipEvent_t ev[4] = {};
    int last_inst = 0;            // instances of the last eig launch (rsp_music_fast_count)
};

namespace {

#define MUCHK(expr)                                                                                    \
    do {                                                                                               \
        hipError_t e_ = (expr);                                                                        \
        if (e_ != hipSuccess)                                                                          \
            return rsp_set_error(RSP_ERR_DEVICE, "%s failed: %s (%s:%d)", #expr, hipGetErrorString(e_), \
                                 __FILE__, __LINE__);                                                  \
    } while (0)

// What a launch's caller reads (music_run): only the peak indices (the block-power fast path may
// replace the eigen-decomposition), also the pseudo-spectrum (full path: the spectrum is then the
// eigensolver's to rounding), or also all N eigenvalues (full path, every eigenvalue).
enum MusicWant { MU_WANT_PEAKS = 0, MU_WANT_SPECTRUM = 1, MU_WANT_EIGS = 2 };

template <int MC>
hipError_t launch_eig64(rsp_music_plan* p, int n_inst, int want) {
    const size_t lds = me_lds_bytes(MC, p->S);
    // neig: eigenvalues the kernel finds (all N when the caller reads them, else the M signal ones)
    const int neig = want == MU_WANT_EIGS ? p->N : p->M;
    // the fast-path instantiation for peaks-only and spectrum calls: a call that reads the
    // eigenvalues never takes it, whatever N and M are (an N <= 4 plan asks for neig = N <= 4 too)
    const bool fast = (want == MU_WANT_PEAKS || want == MU_WANT_SPECTRUM) && MC <= 4;
    // spectrum calls keep the fast subspace only where it bounds P_dB's error by 1e-8 dB
    const double spec_tol = want == MU_WANT_SPECTRUM ? 1e-8 : 0.0;
    const void* kf = fast ? reinterpret_cast<const void*>(k_music_eig64<MC, true>)
                          : reinterpret_cast<const void*>(k_music_eig64<MC, false>);
    if (lds > 64 * 1024) {
        hipError_t e = hipFuncSetAttribute(kf, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        if (e != hipSuccess) return e;
    }
    if (fast)
        hipLaunchKernelGGL((k_music_eig64<MC, true>), dim3(n_inst), dim3(ME_THREADS), lds, p->stream, p->N, p->S, neig,
                           spec_tol, (const double2*)p->d_R, (const double2*)p->d_S1T, p->Spad, (double*)p->d_spec,
                           (double*)p->d_eig, p->d_peaks, p->d_trace);
    else
        hipLaunchKernelGGL((k_music_eig64<MC, false>), dim3(n_inst), dim3(ME_THREADS), lds, p->stream, p->N, p->S,
                           neig, 0.0, (const double2*)p->d_R, (const double2*)p->d_S1T, p->Spad, (double*)p->d_spec,
                           (double*)p->d_eig, p->d_peaks, p->d_trace);
    return hipGetLastError();
}

// want (MusicWant): MU_WANT_EIGS computes every eigenvalue (the caller reads them); otherwise only
// the M signal eigenvalues the vectors and the spectrum need (complex double), and MU_WANT_PEAKS
// allows the fast path
int music_run(rsp_music_plan* p, const void* dX, int n_inst, bool timed, float* ms, int want) {
    if (n_inst < 1 || n_inst > p->max_batch)
        return rsp_set_error(RSP_ERR_INVALID, "n_inst %d outside 1..max_batch %d", n_inst, p->max_batch);
    MUCHK(hipSetDevice(p->device));
    if (timed) MUCHK(hipEventRecord(p->ev[0], p->stream));
    if (p->f64)
        hipLaunchKernelGGL(k_music_cov64, dim3(n_inst), dim3(MU_THREADS), 0, p->stream, p->N, p->K,
                           (const double2*)dX, (double2*)p->d_R);
    else if (p->N % 4 == 0)
        hipLaunchKernelGGL(k_music_cov<true>, dim3(n_inst), dim3(MU_THREADS), 0, p->stream, p->N, p->K,
                           (const float2*)dX, (float2*)p->d_R);
    else
        hipLaunchKernelGGL(k_music_cov<false>, dim3(n_inst), dim3(MU_THREADS), 0, p->stream, p->N, p->K,
                           (const float2*)dX, (float2*)p->d_R);
    MUCHK(hipGetLastError());
    if (timed) MUCHK(hipEventRecord(p->ev[1], p->stream));
    p->last_inst = n_inst;
    if (p->f64) {
        switch (p->M) {
#define MU_EIG64(MC) \
    case MC: MUCHK(launch_eig64<MC>(p, n_inst, want)); break;
            MU_EIG64(1) MU_EIG64(2) MU_EIG64(3) MU_EIG64(4) MU_EIG64(5) MU_EIG64(6) MU_EIG64(7) MU_EIG64(8)
#undef MU_EIG64
        }
    } else {
        switch (p->M) {
#define MU_EIG(MC)                                                                                               \
    case MC:                                                                                                     \
        hipLaunchKernelGGL(k_music_eig<MC>, dim3(n_inst), dim3(64), mu_eig_lds_bytes(MC), p->stream, p->N, p->S, \
                           (const float2*)p->d_R, (const float2*)p->d_S1T, p->Spad, (float*)p->d_spec,            \
                           (float*)p->d_eig, p->d_peaks, p->d_trace);                                             \
        break;
            MU_EIG(1) MU_EIG(2) MU_EIG(3) MU_EIG(4) MU_EIG(5) MU_EIG(6) MU_EIG(7) MU_EIG(8)
#undef MU_EIG
        }
    }
    MUCHK(hipGetLastError());
    if (timed) {
        MUCHK(hipEventRecord(p->ev[2], p->stream));
        MUCHK(hipEventSynchronize(p->ev[2]));
        MUCHK(hipEventElapsedTime(&ms[0], p->ev[0], p->ev[1]));
        MUCHK(hipEventElapsedTime(&ms[1], p->ev[1], p->ev[2]));
    }
    return RSP_OK;
}

// device results -> caller (double; a complex-single plan's are widened)
int music_fetch(rsp_music_plan* p, int n_inst, rsp_music_out* out) {
    if (!out) return RSP_OK;
    const int N = p->N, M = p->M, S = p->S;
    const size_t rs = p->f64 ? 8 : 4;
    std::vector<unsigned char> spec, eig, rc;
    if (out->spectrum_db) {
        if (p->f64)
            MUCHK(hipMemcpyAsync(out->spectrum_db, p->d_spec, (size_t)n_inst * S * 8, hipMemcpyDeviceToHost, p->stream));
        else {
            spec.resize((size_t)n_inst * S * rs);
            MUCHK(hipMemcpyAsync(spec.data(), p->d_spec, spec.size(), hipMemcpyDeviceToHost, p->stream));
        }
    }
    if (out->eigenvalues) {
        if (p->f64)
            MUCHK(hipMemcpyAsync(out->eigenvalues, p->d_eig, (size_t)n_inst * N * 8, hipMemcpyDeviceToHost, p->stream));
        else {
            eig.resize((size_t)n_inst * N * rs);
            MUCHK(hipMemcpyAsync(eig.data(), p->d_eig, eig.size(), hipMemcpyDeviceToHost, p->stream));
        }
    }
    std::vector<int> pk;
    if (out->peak_idx || out->n_peaks) {
        pk.resize((size_t)n_inst * (MU_MMAX + 1));
        MUCHK(hipMemcpyAsync(pk.data(), p->d_peaks, pk.size() * sizeof(int), hipMemcpyDeviceToHost, p->stream));
    }
    if (out->covariance) {
        rc.resize((size_t)n_inst * MU_NMAX * MU_NMAX * 2 * rs);
        MUCHK(hipMemcpyAsync(rc.data(), p->d_R, rc.size(), hipMemcpyDeviceToHost, p->stream));
    }
    MUCHK(hipStreamSynchronize(p->stream));
    if (!spec.empty())
        for (size_t e = 0; e < (size_t)n_inst * S; ++e) out->spectrum_db[e] = reinterpret_cast<const float*>(spec.data())[e];
    if (!eig.empty())
        for (size_t e = 0; e < (size_t)n_inst * N; ++e) out->eigenvalues[e] = reinterpret_cast<const float*>(eig.data())[e];
    for (int i = 0; i < n_inst && !pk.empty(); ++i) {
        if (out->n_peaks) out->n_peaks[i] = pk[(size_t)i * (MU_MMAX + 1)];
        if (out->peak_idx)
            for (int m = 0; m < M; ++m) out->peak_idx[(size_t)i * M + m] = pk[(size_t)i * (MU_MMAX + 1) + 1 + m];
    }
    if (out->covariance)   // N x N column-major complex double per instance
        for (int i = 0; i < n_inst; ++i)
            for (int b = 0; b < N; ++b)
                for (int a = 0; a < N; ++a) {
                    const size_t e = (size_t)i * MU_NMAX * MU_NMAX + a + MU_NMAX * b;
                    double* o = out->covariance + 2 * ((size_t)i * N * N + a + (size_t)N * b);
                    if (p->f64) {
                        const double* v = reinterpret_cast<const double*>(rc.data()) + 2 * e;
                        o[0] = v[0];
                        o[1] = v[1];
                    } else {
                        const float* v = reinterpret_cast<const float*>(rc.data()) + 2 * e;
                        o[0] = v[0];
                        o[1] = v[1];
                    }
                }
    return RSP_OK;
}

}  // namespace

extern "C" {

int32_t rsp_music_create(const rsp_music_config* cfg, int32_t device, rsp_music_plan** out) {
    if (!cfg || !out || !cfg->scan_rad) return rsp_set_error(RSP_ERR_INVALID, "null argument");
    *out = nullptr;
    const int N = cfg->channel_num, K = cfg->num_snapshots, M = cfg->num_sources, S = cfg->n_scan;
    if (N < 2 || N > MU_NMAX) return rsp_set_error(RSP_ERR_UNSUPPORTED, "channel_num %d outside 2..%d", N, MU_NMAX);
    if (M < 1 || M >= N || M > MU_MMAX)
        return rsp_set_error(RSP_ERR_UNSUPPORTED, "num_sources %d outside 1..min(%d, channel_num-1)", M, MU_MMAX);
    if (K < 1) return rsp_set_error(RSP_ERR_INVALID, "num_snapshots %d < 1", K);
    if (S < 3 || S > MU_SCAN_MAX) return rsp_set_error(RSP_ERR_UNSUPPORTED, "n_scan %d outside 3..%d", S, MU_SCAN_MAX);
    if (cfg->max_batch < 1) return rsp_set_error(RSP_ERR_INVALID, "max_batch %d < 1", cfg->max_batch);
    if (cfg->precision != RSP_C128 && cfg->precision != RSP_C64)
        return rsp_set_error(RSP_ERR_INVALID, "precision must be RSP_C128 or RSP_C64, got %d", cfg->precision);
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev)
        return rsp_set_error(RSP_ERR_DEVICE, "HIP device %d not available (%d devices)", device, ndev);
    rsp_music_plan* p = new rsp_music_plan();
    p->device = device;
    p->N = N; p->K = K; p->M = M; p->S = S; p->Spad = (S + 7) & ~3;
    p->max_batch = cfg->max_batch;
    p->dl = cfg->d_over_lambda;
    p->f64 = cfg->precision == RSP_C128;
    p->xsz = p->f64 ? 16 : 8;
    auto bail = [&](int rc) { rsp_music_destroy(p); return rc; };
    if (hipSetDevice(device) != hipSuccess) return bail(rsp_set_error(RSP_ERR_DEVICE, "hipSetDevice(%d)", device));
    if (hipStreamCreateWithFlags(&p->stream, hipStreamNonBlocking) != hipSuccess)
        return bail(rsp_set_error(RSP_ERR_DEVICE, "hipStreamCreate failed"));
    for (auto& e : p->ev)
        if (hipEventCreate(&e) != hipSuccess) return bail(rsp_set_error(RSP_ERR_DEVICE, "hipEventCreate failed"));
    const size_t B = (size_t)p->max_batch, cs = p->xsz, rs = p->xsz / 2;
    struct { void** ptr; size_t bytes; } allocs[] = {
        {&p->d_S1T, (size_t)MU_NMAX * p->Spad * cs},
        {&p->d_R, B * MU_NMAX * MU_NMAX * cs},
        {&p->d_spec, B * S * rs},
        {&p->d_eig, B * N * rs},
        {(void**)&p->d_peaks, B * (MU_MMAX + 1) * sizeof(int)},
        {(void**)&p->d_src, (size_t)MU_MMAX * MU_NMAX * sizeof(double2)},
        {(void**)&p->d_amp, (size_t)MU_MMAX * sizeof(double)},
    };
    for (auto& a : allocs)
        if (hipMalloc(a.ptr, a.bytes) != hipSuccess)
            return bail(rsp_set_error(RSP_ERR_NOMEM, "hipMalloc(%zu bytes) failed", a.bytes));
    // S1 = exp(1j k z sin(phi_list')) (MUSIC_1D.m:36) in double (rounded to float for a complex-single
    // plan); stored transposed [channel][angle]
    std::vector<double2> s1((size_t)MU_NMAX * p->Spad, make_double2(0.0, 0.0));
    for (int c = 0; c < N; ++c)
        for (int s = 0; s < S; ++s) {
            const double ph = 2.0 * M_PI * p->dl * c * std::sin(cfg->scan_rad[s]);
            s1[(size_t)c * p->Spad + s] = make_double2(std::cos(ph), std::sin(ph));
        }
    hipError_t e;
    if (p->f64) {
        e = hipMemcpy(p->d_S1T, s1.data(), s1.size() * sizeof(double2), hipMemcpyHostToDevice);
    } else {
        std::vector<float2> s1f(s1.size());
        for (size_t i = 0; i < s1.size(); ++i) s1f[i] = make_float2((float)s1[i].x, (float)s1[i].y);
        e = hipMemcpy(p->d_S1T, s1f.data(), s1f.size() * sizeof(float2), hipMemcpyHostToDevice);
    }
    if (e != hipSuccess) return bail(rsp_set_error(RSP_ERR_DEVICE, "steering upload failed"));
#ifdef RSP_DEBUG_KNOBS   // diagnostic builds only: the shipped library reads no environment variable
    const char* tr = getenv("RSP_MUSIC_TRACE");
    if (tr && atoi(tr) && hipMalloc(&p->d_trace, B * 8 * sizeof(unsigned long long)) != hipSuccess)
        return bail(rsp_set_error(RSP_ERR_NOMEM, "trace buffer"));
#endif
    *out = p;
    return RSP_OK;
}

int32_t rsp_music_destroy(rsp_music_plan* p) {
    if (!p) return RSP_OK;
    (void)hipSetDevice(p->device);
    if (p->stream) (void)hipStreamSynchronize(p->stream);
    void* bufs[] = {p->d_S1T, p->d_R, p->d_X, p->d_spec, p->d_eig, p->d_peaks, p->d_src, p->d_amp, p->d_trace};
    for (void* b : bufs)
        if (b) (void)hipFree(b);
    for (auto& e : p->ev)
        if (e) (void)hipEventDestroy(e);
    if (p->stream) (void)hipStreamDestroy(p->stream);
    delete p;
    return RSP_OK;
}

int32_t rsp_music_synthesize_device(rsp_music_plan* p, const rsp_music_scene* sc, int32_t n_inst, int32_t inst0,
                                    uint64_t seed, void* d_X) {
    if (!p || !sc || !d_X) return rsp_set_error(RSP_ERR_INVALID, "null argument");
    if (sc->n_src < 1 || sc->n_src > MU_MMAX)
        return rsp_set_error(RSP_ERR_UNSUPPORTED, "n_src %d outside 1..%d", sc->n_src, MU_MMAX);
    if (n_inst < 1) return rsp_set_error(RSP_ERR_INVALID, "n_inst %d < 1", n_inst);
    MUCHK(hipSetDevice(p->device));
    const int N = p->N, Ms = sc->n_src;
    std::vector<double2> src((size_t)Ms * N);
    for (int m = 0; m < Ms; ++m)   // S = exp(1j k z sin(phi')) (MUSIC_1D.m:21)
        for (int c = 0; c < N; ++c) {
            const double ph = 2.0 * M_PI * p->dl * c * std::sin(sc->angles_rad[m]);
            src[(size_t)m * N + c] = make_double2(std::cos(ph), std::sin(ph));
        }
    double amp[MU_MMAX];
    for (int m = 0; m < MU_MMAX; ++m) amp[m] = m < Ms ? sc->amplitudes[m] : 0.0;
    MUCHK(hipMemcpyAsync(p->d_src, src.data(), src.size() * sizeof(double2), hipMemcpyHostToDevice, p->stream));
    MUCHK(hipMemcpyAsync(p->d_amp, amp, sizeof amp, hipMemcpyHostToDevice, p->stream));
    const double nsc_fixed = std::sqrt(1.0 / std::pow(10.0, sc->snr_db / 10.0) / 2.0);
    if (p->f64)
        hipLaunchKernelGGL(k_music_synth<double2>, dim3(n_inst), dim3(MU_THREADS), 0, p->stream, N, p->K, Ms, inst0,
                           seed, p->d_src, p->d_amp, sc->complex_sources, sc->snr_measured ? 1 : 0, sc->snr_db,
                           nsc_fixed, (double2*)d_X);
    else
        hipLaunchKernelGGL(k_music_synth<float2>, dim3(n_inst), dim3(MU_THREADS), 0, p->stream, N, p->K, Ms, inst0,
                           seed, p->d_src, p->d_amp, sc->complex_sources, sc->snr_measured ? 1 : 0, sc->snr_db,
                           nsc_fixed, (float2*)d_X);
    MUCHK(hipGetLastError());
    MUCHK(hipStreamSynchronize(p->stream));   // the host staging above is stack memory
    return RSP_OK;
}

int32_t rsp_music_process_device(rsp_music_plan* p, const void* d_X, int32_t n_inst, rsp_music_out* out) {
    if (!p || !d_X) return rsp_set_error(RSP_ERR_INVALID, "null argument");
    const int want = !out ? MU_WANT_PEAKS
                          : out->eigenvalues ? MU_WANT_EIGS : out->spectrum_db ? MU_WANT_SPECTRUM : MU_WANT_PEAKS;
    int rc = music_run(p, d_X, n_inst, false, nullptr, want);
    if (rc) return rc;
    if (!out) {
        MUCHK(hipStreamSynchronize(p->stream));
        return RSP_OK;
    }
    return music_fetch(p, n_inst, out);
}

int32_t rsp_music_process(rsp_music_plan* p, const void* X, int32_t dtype, int32_t n_inst, rsp_music_out* out) {
    if (!p || !X) return rsp_set_error(RSP_ERR_INVALID, "null argument");
    if (n_inst < 1 || n_inst > p->max_batch)
        return rsp_set_error(RSP_ERR_INVALID, "n_inst %d outside 1..max_batch %d", n_inst, p->max_batch);
    if (dtype != RSP_C64 && dtype != RSP_C128) return rsp_set_error(RSP_ERR_INVALID, "unknown dtype %d", dtype);
    MUCHK(hipSetDevice(p->device));
    const size_t elems = (size_t)n_inst * p->K * p->N;
    if (!p->d_X) {
        const size_t bytes = (size_t)p->max_batch * p->K * p->N * p->xsz;
        if (hipMalloc(&p->d_X, bytes) != hipSuccess)
            return rsp_set_error(RSP_ERR_NOMEM, "hipMalloc(%zu bytes) failed", bytes);
    }
    if ((dtype == RSP_C128) == p->f64) {
        MUCHK(hipMemcpy(p->d_X, X, elems * p->xsz, hipMemcpyHostToDevice));
    } else if (p->f64) {   // complex single snapshots into a complex-double plan: widen
        std::vector<double2> h(elems);
        const float* x = (const float*)X;
        for (size_t i = 0; i < elems; ++i) h[i] = make_double2(x[2 * i], x[2 * i + 1]);
        MUCHK(hipMemcpy(p->d_X, h.data(), elems * sizeof(double2), hipMemcpyHostToDevice));
    } else {
        std::vector<float2> h(elems);
        const double* x = (const double*)X;
        for (size_t i = 0; i < elems; ++i) h[i] = make_float2((float)x[2 * i], (float)x[2 * i + 1]);
        MUCHK(hipMemcpy(p->d_X, h.data(), elems * sizeof(float2), hipMemcpyHostToDevice));
    }
    return rsp_music_process_device(p, p->d_X, n_inst, out);
}

int32_t rsp_music_profile(rsp_music_plan* p, const void* d_X, int32_t n_inst, int32_t iters, float* ms_out) {
    return rsp_music_profile_ex(p, d_X, n_inst, iters, RSP_MUSIC_PEAKS, ms_out);
}

int32_t rsp_music_profile_ex(rsp_music_plan* p, const void* d_X, int32_t n_inst, int32_t iters, int32_t what,
                             float* ms_out) {
    if (!p || !d_X || !ms_out || iters < 1) return rsp_set_error(RSP_ERR_INVALID, "bad argument");
    if (what != RSP_MUSIC_PEAKS && what != RSP_MUSIC_SPECTRUM && what != RSP_MUSIC_EIGENVALUES)
        return rsp_set_error(RSP_ERR_INVALID, "unknown profile form %d", what);
    const int want = what == RSP_MUSIC_EIGENVALUES ? MU_WANT_EIGS
                   : what == RSP_MUSIC_SPECTRUM ? MU_WANT_SPECTRUM : MU_WANT_PEAKS;
    double acc[2] = {0.0, 0.0};
    for (int it = 0; it < iters; ++it) {
        float ms[2];
        int rc = music_run(p, d_X, n_inst, true, ms, want);
        if (rc) return rc;
        acc[0] += ms[0];
        acc[1] += ms[1];
    }
    ms_out[0] = (float)(acc[0] / iters);
    ms_out[1] = (float)(acc[1] / iters);
    if (p->d_trace) {   // mean phase durations of the last launch (s_memrealtime: 100 MHz)
        std::vector<unsigned long long> t((size_t)n_inst * 8);
        MUCHK(hipMemcpy(t.data(), p->d_trace, t.size() * sizeof(t[0]), hipMemcpyDeviceToHost));
        double ph[6] = {0, 0, 0, 0, 0, 0};
        for (int i = 0; i < n_inst; ++i)
            for (int q = 0; q < 6; ++q) ph[q] += (double)(t[(size_t)i * 8 + q + 1] - t[(size_t)i * 8 + q]) * 0.01 / n_inst;
        double tf = 0;   // stamp 7 (complex double): dlagtf's end, inside the inverse-iteration phase
        for (int i = 0; i < n_inst && p->f64; ++i) tf += (double)(t[(size_t)i * 8 + 7] - t[(size_t)i * 8 + 2]) * 0.01 / n_inst;
        fprintf(stderr, "k_music_eig%s phases (us/instance): tridiag %.2f eigenvalues %.2f inviter %.2f (dlagtf %.2f) backxf %.2f spectrum %.2f peaks %.2f\n",
                p->f64 ? "64" : "",
                ph[0], ph[1], ph[2], tf, ph[3], ph[4], ph[5]);
    }
    return RSP_OK;
}

int32_t rsp_music_device_alloc(rsp_music_plan* p, int64_t bytes, void** d_ptr) {
    if (!p || !d_ptr || bytes <= 0) return rsp_set_error(RSP_ERR_INVALID, "bad argument");
    MUCHK(hipSetDevice(p->device));
    if (hipMalloc(d_ptr, (size_t)bytes) != hipSuccess)
        return rsp_set_error(RSP_ERR_NOMEM, "hipMalloc(%lld bytes) failed", (long long)bytes);
    return RSP_OK;
}

int32_t rsp_music_device_free(rsp_music_plan* p, void* d_ptr) {
    if (!p) return rsp_set_error(RSP_ERR_INVALID, "null plan");
    MUCHK(hipSetDevice(p->device));
    MUCHK(hipStreamSynchronize(p->stream));
    MUCHK(hipFree(d_ptr));
    return RSP_OK;
}

int32_t rsp_music_fast_count(rsp_music_plan* p, int32_t* n_fast) {
    if (!p || !n_fast) return rsp_set_error(RSP_ERR_INVALID, "bad argument");
    *n_fast = 0;
    if (!p->f64 || p->M >= MU_MMAX || p->last_inst < 1) return RSP_OK;   // only complex double, M <= 4, sets it
    MUCHK(hipSetDevice(p->device));
    MUCHK(hipStreamSynchronize(p->stream));
    std::vector<int> pk((size_t)p->last_inst * (MU_MMAX + 1));
    MUCHK(hipMemcpy(pk.data(), p->d_peaks, pk.size() * sizeof(int), hipMemcpyDeviceToHost));
    for (int i = 0; i < p->last_inst; ++i) *n_fast += pk[(size_t)i * (MU_MMAX + 1) + MU_MMAX] == 1;
    return RSP_OK;
}

int32_t rsp_music_device_download(rsp_music_plan* p, void* h_dst, const void* d_src, int64_t bytes) {
    if (!p || !h_dst || !d_src || bytes < 0) return rsp_set_error(RSP_ERR_INVALID, "bad argument");
    MUCHK(hipSetDevice(p->device));
    MUCHK(hipStreamSynchronize(p->stream));
    MUCHK(hipMemcpy(h_dst, d_src, (size_t)bytes, hipMemcpyDeviceToHost));
    return RSP_OK;
}

}  // extern "C"
