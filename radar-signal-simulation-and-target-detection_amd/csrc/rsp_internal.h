// rsp_internal.h -- shared host/device descriptors of librsp (not part of the C-ABI).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define RSP_MAX_F 8          // frames batched per launch
#define RSP_LANES 4          // max streams of the throughput queue (batches in flight)
#define RSP_NLANES 3         // streams the throughput queue uses (<= RSP_LANES)
#define RSP_K2_POINTS 4096   // complex points per pulse-compression workgroup (Geometry::k2_pts)
#define RSP_K2_MIXPTS 2560   // Geometry::k2_pts of a complex-double plan with a 2560-point block
#define K2_THREADS 256       // threads per pulse-compression workgroup (16 points each)
#define RSP_THREADS 256
// The kernel variants measured and not kept (profiles/EXPERIMENTS.md) were removed in round 6;
// the library has one code path per configuration and no compile-time A/B switches.

// Arithmetic of a plan: every device buffer, table and operation of the chain is in one of
// these.  PREC_F64 is MATLAB's complex double (the reference's arithmetic, fsf:47,92,101,131);
// PREC_F32 is complex single (an explicitly narrower option).
#define RSP_PREC_F32 0
#define RSP_PREC_F64 1

// Philox4x32-10 (Salmon et al., SC'11) in place on counter c with key (k0, k1); the streams
// built on it are documented in oracle/philox.py (echo noise) and oracle/music.py (MUSIC).
__device__ __forceinline__ void rsp_philox10(uint32_t c[4], uint32_t k0, uint32_t k1) {
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

// Device record of one CFAR detection + its S9 estimate; layout == rsp_detection.
struct DevDet {
    int32_t v_idx, r_idx, pair_idx, reserved;   // 1-based like fsf:220
    double amp, range, velocity, angle;
};

// Pulse-compression segment (fsf:105-126).  Output gates [ga, gb) of the stitched
// row come from this segment.  x~(n) = x(n) for lo_eff <= n <= hi, else 0, where
// [lo, hi] is the window of samples that reach a kept gate (plan-time analysis).
struct SegDesc {
    int type;        // 0 = direct FIR (narrow, fsf:111-112), 1 = FFT overlap-save (fsf:115-120)
    int ga, gb;      // stitched gate range
    int seg_lo;      // 0-based first sample of the segment (seg_start - 1)
    int lo, hi;      // needed sample window (0-based, inclusive), lo >= seg_lo
    int off;         // compacted sample index of `lo`
    // direct FIR: y[g] = sum_j h[j] x~(seg_lo + k - j), k = (g + delay) mod Ls
    int ntaps, delay, Ls, taps_off;
    // FFT overlap-save: y[g] = sum_{j<Lh} h[j] x~(seg_lo + g - j), block size M = 2^logM,
    // V = M-Lh+1 valid outputs per block
    int Lh, M, logM, V, nblocks, H_off, tw_off;
    int rows_per_wg;
};

// One group of pulse-compression workgroups: segment `seg`, overlap-save block `blk`.
struct K2Job {
    int seg, blk, wg_begin, wg_count;
};

#define RSP_MAX_SEG 3
#define RSP_MAX_JOBS 16
#define RSP_MAX_IVL 4

struct Geometry {
    int prec;        // RSP_PREC_F32 / RSP_PREC_F64
    int C, B, P, N, G;
    int cpitch;      // device cube channel pitch in complex samples (= N*P)
    int Gp;          // row stride of the magnitude maps (G rounded up to 4)
    int NT, nU, ntiles, Ppad;
    int NZ, nzc;     // z layout: NZ compacted samples per (row, chunk) slab, nzc chunks per row
    int twPp_elems;  // per-pass twiddles of the P-point FFT
    int pow2P, logP;
    // non-power-of-two P = rqR * rqQ (rqR = 2 or 4, rqQ odd >= 3): K1's factored slow-time DFT
    // (k1_dft_rq); rqQ = 0: the direct O(P^2) DFT.  twq_elems = complex entries of its
    // frequency-set twiddle table (DevConsts::twQ)
    int rqR, rqQ, twq_elems;
    int nseg, njobs, nwg_k2;
    // complex points of LDS rows per pulse-compression workgroup: RSP_K2_POINTS, or 2560 in a
    // complex-double plan with a 2560-point block (4 workgroups per CU: 40 KB of LDS each, no pads);
    // power-of-two blocks then take 2048 / M rows
    int k2_pts;
    int cfar_RT, cfar_hR, cfar_W;
    int cfar_VB, cfar_nband, cfar_rows;   // K3 Doppler bands: cells under test per band, bands, tile rows
    int refR, guardR, refV, guardV;
    double T;        // T_CFAR
    int max_dets;    // detection-list capacity per frame of the launch (grows on demand, rsp_plan.cpp)
    int ncu;         // compute units of the device (persistent K1 grid)
    int k1_tiled;    // force the one-tile-per-workgroup K1 (RSP_PLAN_K1_TILED, parity tests)
    int mono_c;      // S9 angle from the complex ratio of the RD map (RSP_PLAN_MONOPULSE_COMPLEX)
    // used fast-time samples as <= RSP_MAX_IVL intervals: compacted n' in [ivl_start[q],
    // ivl_start[q+1]) is sample ivl_lo[q] + n' - ivl_start[q] (kernel-argument lookup, no
    // dependent global load before the cube loads)
    int nivl, ivl_lo[RSP_MAX_IVL], ivl_start[RSP_MAX_IVL];
    // pulse-compression segment and job tables travel as kernel arguments too
    SegDesc segs[RSP_MAX_SEG];
    K2Job jobs[RSP_MAX_JOBS];
};

// K3's compile-time path: the reference's cfar_params (v8:45-46) and a 32/64-cell tile
__host__ __device__ inline bool k3_fast_params(const Geometry& g) {
    return g.refR == 5 && g.refV == 5 && g.guardR == 10 && g.guardV == 10 && (g.cfar_RT == 32 || g.cfar_RT == 64);
}

// K3 tiles: range cells from the first cell under test rounded down to 4, cfar_RT per tile
// (k3_cfar, launch_k3, rsp_profile_stages).
__host__ __device__ inline int k3_ntiles(const Geometry& g) {
    const int rc0 = g.refR + g.guardR;
    return (g.G - rc0 - (rc0 & ~3) + g.cfar_RT - 1) / g.cfar_RT;
}

// Magnitude-map bytes K3 reads from HBM per frame (the K3 stage's algorithmic bytes): on the
// fast path the halo-less tiles hold only the Doppler rows under test, P - 2 (refV + guardV), over
// the tiled range columns (first cell under test rounded down to 4, k3_ntiles * cfar_RT cells,
// clipped to G); each beam's map is read by two pairs, the second read an L2 hit (XCD-aware
// order).  The general path reads whole maps.  bench.py / tests/test_bench_args.py restate it.
__host__ __device__ inline long long k3_map_bytes(const Geometry& g, int real_bytes) {
    if (k3_fast_params(g)) {
        const int hV = g.refV + g.guardV, c0 = (g.refR + g.guardR) & ~3;
        const int rows = g.P - 2 * hV > 0 ? g.P - 2 * hV : 0;
        const int c1 = c0 + k3_ntiles(g) * g.cfar_RT < g.G ? c0 + k3_ntiles(g) * g.cfar_RT : g.G;
        return (long long)g.B * rows * (c1 > c0 ? c1 - c0 : 0) * real_bytes;
    }
    return (long long)g.B * g.P * g.G * real_bytes;
}

// Per-frame device buffers of one launch.  Element types follow Geometry::prec: complex
// values are (re, im) pairs of float or double, maps are float or double.
struct FramePtrs {
    const void* in[RSP_MAX_F];     // K1 input cube (PNC) or beam cube
    void* z[RSP_MAX_F];            // compacted Doppler-domain rows
    void* rdm[RSP_MAX_F];          // [B][P][G] complex
    void* mag[RSP_MAX_F];          // |rdm| [B][P][Gp] (K2 epilogue, read by K3)
    void* smap[RSP_MAX_F];         // optional: rdm_for_cfar_all [B-1][P][G] as K3 thresholds it (fsf:184-187)
    unsigned long long* trace;     // diagnostic builds (-DRSP_DEBUG_KNOBS): 4 stamps per workgroup
    DevDet* dets[RSP_MAX_F];
    int* count[RSP_MAX_F];
};

struct DevConsts {
    const void* Atab;        // DBF MFMA A operands per lane: [MB][CP/4][Re,Im][64] (build_dbf_atab), real
    const void* win;         // MTD window [P], real
    const void* twP;         // W_P^i table (direct DFT path), complex
    const void* twPp;        // per-pass Stockham twiddles of the P-point FFT, complex
    const void* twD;         // persistent K1's in-place FFT: [i][n2] = W_P^(n2 2^i), i < 4, n2 < P/16, complex
    const void* twQ;         // factored DFT (P = R Q): [fset][n - 1][r] = (cos, sin)(2 pi k n / Q), k = RQ_RK fset + r
    const void* taps;        // narrow FIR taps, real
    const void* H;           // overlap-save spectra, 1/M scaled, complex
    const void* twM;         // per-pass Stockham twiddles of each overlap-save block size, complex
    const int* k2order;      // pulse-compression workgroup dispatch order: job kinds interleaved
    const double* range_axis;
    const double* velocity_axis;
    const double* beam_angles;
    const double* klut;
    double deltaR, deltaV;
};

struct SynthTarget {          // per-target constants of S4 (fsf:51-73), host-computed
    int delay;                // delay_samples
    double amp;
    double fd_prt;            // doppler_freq * prt   (phase per pulse / 2pi)
    double dphi;              // channel phase step (rad)
};
#define RSP_MAX_SYNTH_TARGETS 64
struct SynthTargets {         // by value in the kernel arguments (2 KiB): no upload, no sync
    SynthTarget t[RSP_MAX_SYNTH_TARGETS];
};

// Frequencies per wave-uniform set of the factored slow-time DFT's Q-point stage (k1_dft_rq)
#define RQ_RK 6

// Launchers (rsp_kernels.hip).  `mode` bits for K1: 1 = apply DBF, 2 = apply MTD.
hipError_t launch_k1(const Geometry& g, const DevConsts& k, const FramePtrs& fp, int nf, int mode, hipStream_t s);
hipError_t launch_stream_copy(const void* in, void* out, size_t n16, int ncu, hipStream_t s);
hipError_t launch_k2(const Geometry& g, const DevConsts& k, const FramePtrs& fp, int nf, int rows, hipStream_t s);
hipError_t launch_k3(const Geometry& g, const DevConsts& k, const FramePtrs& fp, int nf, hipStream_t s);
hipError_t launch_mtd_cols(const Geometry& g, const DevConsts& k, const void* pc, void* rdm, hipStream_t s);
// S4 + S4.1: tab holds RSP_MAX_SYNTH_TARGETS x (P + C) complex doubles (the per-target phasors)
hipError_t launch_synth(const Geometry& g, const double* tx, const SynthTargets& tg, int nt, void* tab, int frame_idx,
                        uint64_t seed, double noise_scale, void* cube, hipStream_t s);
// Queue read-back: count record + the detections of nf frames (device stride dcap + 1 records) into
// mapped pinned host memory (stride hcap + 1), only the records that exist.
hipError_t launch_dets_to_host(const void* dets, int dcap, void* host, int hcap, int nf, hipStream_t s);
// K1 tile geometry the launcher will use (persistent or tiled) for the plan's NT choice
bool k1_persistent_fits(const Geometry& g);
