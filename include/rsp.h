/*
 * rsp.h -- C-ABI of the MI355X radar signal-processing library (librsp.so).
 *
 * Drop-in boundary for the per-frame chain of the MATLAB reference
 * (XuZerui2023/Radar-Signal-Simulation-and-Target-Detection, Simulation/):
 *
 *   final_targets = fun_process_single_frame(targets, config, cfar_params,
 *                       cluster_params, precomputed_data, frame_idx)
 *                                              (fun_process_single_frame.m:13)
 *   [MTD_results, PC_results] = process_stage2_mtd(iq_data, angle, config)
 *                                              (process_stage2_mtd.m:1)
 *
 * The reference has no FFI; these entry points are what a MEX gateway or a
 * MATLAB `loadlibrary`/`calllib` binding of that path binds.
 * Plain C types only: pointers, sizes, int32 status codes.
 *
 * Conventions (mirroring MATLAB so a MEX gateway passes mxArray data as is):
 *   - complex arrays are interleaved (re, im) doubles (mxGetComplexDoubles,
 *     R2018a API) or interleaved floats (RSP_C64);
 *   - matrices are column-major; the echo cube is [P x N x C] (pulse fastest),
 *     range-Doppler maps [P x G x B], CFAR maps [P x G x (B-1)];
 *   - indices reported to the caller are 1-based (fun_process_single_frame.m:220);
 *   - segment starts in rsp_precomputed are 1-based (v8:116-117,130).
 * Arithmetic: a plan computes in complex double (RSP_C128, MATLAB's double as in
 * fun_process_single_frame.m:47,92,101,131 -- the default) or, on request, complex
 * single (RSP_C64); device-resident cubes and maps are in the plan's precision.
 * Errors: every function returns RSP_OK (0) or a negative rsp_status; the
 * message of the last failure on the calling thread is rsp_last_error().
 * Threading: a plan is not thread-safe; use one plan per host thread (MATLAB
 * parfor workers are processes, each with its own plan).
 */
#ifndef RSP_H
#define RSP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RSP_ABI_VERSION 4

typedef enum rsp_status {
    RSP_OK = 0,
    RSP_ERR_INVALID = -1,      /* bad argument / inconsistent config            */
    RSP_ERR_UNSUPPORTED = -2,  /* config outside what the kernels implement      */
    RSP_ERR_DEVICE = -3,       /* HIP runtime failure                            */
    RSP_ERR_NOMEM = -4,        /* device or host allocation failed               */
    RSP_ERR_OVERFLOW = -5      /* a caller-sized output buffer is too small      */
} rsp_status;

typedef enum rsp_dtype {
    RSP_C64 = 1,   /* interleaved complex float  */
    RSP_C128 = 2   /* interleaved complex double (MATLAB) */
} rsp_dtype;

typedef enum rsp_layout {
    RSP_LAYOUT_PNC = 0   /* MATLAB column-major [P x N x C]: index m + P*(n + N*c) */
} rsp_layout;

/* config.Sig_Config + config.Array (main_simulate_echoes_with_array_v8.m:54-69). */
typedef struct rsp_sig_config {
    double c;                 /* Sig_Config.c                       */
    double fs;                /* Sig_Config.fs                      */
    double fc;                /* Sig_Config.fc                      */
    double prt;               /* Sig_Config.prt (s)                 */
    double wavelength;        /* Sig_Config.wavelength              */
    double element_spacing;   /* Array.element_spacing (m)          */
    int32_t prtNum;           /* P: pulses per frame                */
    int32_t point_PRT;        /* N: fast-time samples per pulse     */
    int32_t channel_num;      /* C                                  */
    int32_t beam_num;         /* B                                  */
} rsp_sig_config;

/* cfar_params (v8:45-47). Only 'GOCA' exists in the reference. */
typedef struct rsp_cfar_params {
    int32_t refCells_V, guardCells_V, refCells_R, guardCells_R;
    double T_CFAR;
} rsp_cfar_params;

/* cluster_params (v8:49-51). */
typedef struct rsp_cluster_params {
    double max_range_sep, max_vel_sep, max_angle_sep;
} rsp_cluster_params;

/* precomputed_data (v8:79-155).  Arrays are borrowed for rsp_plan_create only. */
typedef struct rsp_precomputed {
    const double* tx_pulse;            /* complex, point_PRT entries (synthesis; may be NULL) */
    double P_signal_unscaled;
    const double* DBF_coeffs_data_C;   /* complex, B x C column-major                        */
    const double* MF_narrow;           /* real FIR taps                                      */
    int32_t n_MF_narrow;
    int32_t fir_delay;
    const double* MF_medium_fft;       /* complex, N_fft_med entries                          */
    int32_t N_fft_med;
    const double* MF_long_fft;         /* complex, N_fft_long entries                         */
    int32_t N_fft_long;
    int32_t N_gate_narrow, N_gate_medium, N_gate_long, N_total_gate;
    int32_t seg_start_narrow, seg_start_medium, seg_start_long;   /* 1-based */
    const double* MTD_win;             /* prtNum                                              */
    const double* range_axis;          /* N_total_gate                                        */
    const double* velocity_axis;       /* prtNum                                              */
    double deltaR, deltaV;
    const double* beam_angles_deg;     /* beam_num                                            */
    const double* k_slopes_LUT;        /* beam_num - 1                                        */
} rsp_precomputed;

/* targets(k) of the driver (v8:29-37). */
typedef struct rsp_target_in {
    double Range, Velocity, ElevationAngle, SNR_dB;
} rsp_target_in;

/* One entry of final_targets / intra_beam_targets (fun_process_single_frame.m:393-406). */
typedef struct rsp_target {
    double Range, Velocity, Angle, Power;
} rsp_target;

/* One row of all_raw_detections (fsf:220, 1-based v/r/pair, the CFAR map value)
 * together with its S9 estimate (fsf:293-297). */
typedef struct rsp_detection {
    int32_t v_idx, r_idx, pair_idx, reserved;
    double amp;
    double Range, Velocity, Angle;
} rsp_detection;

/* Caller-owned outputs of one frame.  Any pointer may be NULL (not produced).
 * Sizes from rsp_query_sizes. */
typedef struct rsp_frame_out {
    double* rdm;              /* complex, [P x G x B] column-major (rdm_13beam, fsf:135)        */
    double* cfar_maps;        /* real, [P x G x (B-1)] (rdm_for_cfar_all, fsf:187)             */
    rsp_detection* dets;      /* parameterized detections in reference order                   */
    int32_t dets_cap;
    int32_t n_dets;           /* out                                                           */
    rsp_target* targets;      /* final_targets                                                 */
    int32_t targets_cap;
    int32_t n_targets;        /* out                                                           */
} rsp_frame_out;

typedef struct rsp_sizes {
    int64_t cube_elems;       /* P*N*C complex samples                      */
    int64_t rdm_elems;        /* P*G*B                                      */
    int64_t cfar_map_elems;   /* P*G*(B-1)                                  */
    int32_t P, N, C, B, G;
    int32_t used_samples;     /* fast-time samples the chain actually reads */
    int32_t max_detections;   /* most detections a frame can have (cells under
                                 test of every beam pair); the device lists
                                 start smaller and grow on demand           */
    int32_t n_stages;         /* device stages (for rsp_profile_stages)     */
    int32_t precision;        /* RSP_C128 or RSP_C64: device cube / map type */
    int32_t elem_bytes;       /* bytes of one device complex element (16/8) */
} rsp_sizes;

typedef struct rsp_plan rsp_plan;

int32_t rsp_abi_version(void);
const char* rsp_last_error(void);

/* Plan options (rsp_plan_options_default fills the defaults shown). */
#define RSP_PLAN_K1_TILED 1   /* force the one-tile-per-workgroup K1 instead of the persistent
                                 one (both compute the same operations; parity tests compare them) */
#define RSP_PLAN_MONOPULSE_COMPLEX 2   /* S9's angle from the complex ratio
                                 real((S_A - S_B) / (S_A + S_B + eps)) of the RD map, as the inline S9
                                 of main_plot_snr_vs_angle_error.m:455-462, instead of fsf:282-290's
                                 amplitude ratio (|S_A| - |S_B|) / (|S_A| + |S_B| + eps).  K2 then
                                 writes every frame's complex RD map (the caller's, or plan-owned) */
typedef struct rsp_plan_options {
    int32_t device;              /* HIP device ordinal (0)                                   */
    int32_t frames_per_launch;   /* frames batched into each kernel launch by the queue (1)  */
    int32_t precision;           /* RSP_C128 (MATLAB double, default) or RSP_C64             */
    int32_t flags;               /* RSP_PLAN_* (0)                                           */
} rsp_plan_options;
int32_t rsp_plan_options_default(rsp_plan_options* opt);

/* Build a plan: uploads DBF weights, FIR taps, matched-filter spectra (re-blocked for
 * overlap-save), MTD window, axes, angles, K-LUT in the plan's precision.
 * `frames_per_launch` (1..8) frames are batched into each kernel launch by the
 * queue interface; rsp_process_* always run one frame.  rsp_plan_create = the defaults
 * with `device` and `frames_per_launch` (complex double). */
int32_t rsp_plan_create_ex(const rsp_sig_config* cfg, const rsp_cfar_params* cfar,
                           const rsp_cluster_params* cluster, const rsp_precomputed* pre,
                           const rsp_plan_options* opt, rsp_plan** out);
int32_t rsp_plan_create(const rsp_sig_config* cfg, const rsp_cfar_params* cfar,
                        const rsp_cluster_params* cluster, const rsp_precomputed* pre,
                        int32_t device, int32_t frames_per_launch, rsp_plan** out);
int32_t rsp_plan_destroy(rsp_plan* plan);
int32_t rsp_query_sizes(const rsp_plan* plan, rsp_sizes* out);

/* Cube-in path: S5..S11 of fun_process_single_frame on one host cube
 * (layout RSP_LAYOUT_PNC, dtype RSP_C64 or RSP_C128; converted to the plan's precision
 * only if they differ).  Synchronous.  out->cfar_maps, when requested, is the map K3
 * thresholds on the device (rdm_for_cfar_all, fsf:184-187). */
int32_t rsp_process_cube(rsp_plan* plan, const void* cube, int32_t dtype, int32_t layout,
                         int32_t frame_idx, rsp_frame_out* out);

/* Every detection of the last synchronous frame (rsp_process_cube / rsp_process_targets), in the
 * reference's order.  A frame's list has no fixed capacity (all_raw_detections(end+1,:),
 * fsf:215-221); a caller that passed out->dets == NULL or a dets_cap below out->n_dets reads the
 * whole list here.  *n = its length; RSP_ERR_OVERFLOW if cap < *n (the first cap are copied). */
int32_t rsp_last_detections(const rsp_plan* plan, rsp_detection* dets, int32_t cap, int32_t* n);
/* The final targets of the last synchronous frame, likewise (for out->targets == NULL or a
 * targets_cap below out->n_targets). */
int32_t rsp_last_targets(const rsp_plan* plan, rsp_target* targets, int32_t cap, int32_t* n);

/* Reference-signature path (fsf:13): S4 echo synthesis + S4.1 Philox noise
 * (seed, frame_idx) on the device, then S5..S11.  Needs tx_pulse in the plan. */
int32_t rsp_process_targets(rsp_plan* plan, const rsp_target_in* targets, int32_t n_targets,
                            int32_t frame_idx, uint64_t seed, double p_noise, rsp_frame_out* out);

/* Synthesise (S4 + S4.1) one cube on the device into `d_cube` (the plan's precision,
 * PNC layout, device pointer with cube_elems entries).  Synchronous. */
int32_t rsp_synthesize_device(rsp_plan* plan, const rsp_target_in* targets, int32_t n_targets,
                              int32_t frame_idx, uint64_t seed, double p_noise, void* d_cube);
/* Device time of that synthesis (its two kernels: per-target phasor tables, then the cube),
 * averaged over `iters` back-to-back launches into d_cube, by HIP events on the plan's stream.
 * *bytes_out (may be NULL) = the cube bytes one synthesis writes, C x N x P elements. */
int32_t rsp_profile_synthesis(rsp_plan* plan, const rsp_target_in* targets, int32_t n_targets, int32_t iters,
                              void* d_cube, float* ms_out, int64_t* bytes_out);

/* ---- device-resident queue (throughput path) ----
 * rsp_enqueue_device: process a PNC cube (the plan's precision) already resident in
 * device memory.  Frames are batched frames_per_launch at a time and alternate over the
 * plan's lanes (streams); detections come back asynchronously and are clustered
 * on the host.  rsp_drain waits for everything queued.  Results are kept in
 * enqueue order until rsp_results_clear. */
int32_t rsp_enqueue_device(rsp_plan* plan, const void* d_cube, int32_t frame_idx);
/* rsp_enqueue_device for n frames in one call (d_cubes[i], frame_idx[i]).  All or nothing: a null
 * d_cubes[i] (or d_rdms[i] in the _rdm_n form) is refused before any frame is queued. */
int32_t rsp_enqueue_device_n(rsp_plan* plan, const void* const* d_cubes, const int32_t* frame_idx, int32_t n);
/* rsp_enqueue_device that also produces the frame's complex range-Doppler map rdm_13beam
 * (fsf:131-136, the rsp_mex('cube') output): K2 writes it straight into the caller's device buffer
 * d_rdm (rsp_sizes.rdm_elems complex elements in the plan's precision, device layout [B][P][G],
 * range fastest).  d_rdm must stay allocated, and must not be handed to another frame, until
 * rsp_drain returns; the map is complete then.  Without it (rsp_enqueue_device) the map stays
 * on chip and only |RDM| reaches HBM. */
int32_t rsp_enqueue_device_rdm(rsp_plan* plan, const void* d_cube, int32_t frame_idx, void* d_rdm);
int32_t rsp_enqueue_device_rdm_n(rsp_plan* plan, const void* const* d_cubes, const int32_t* frame_idx,
                                 void* const* d_rdms, int32_t n);
/* End-to-end form of rsp_enqueue_device: a host PNC cube in the plan's precision (no conversion;
 * rsp_process_cube converts).  Only the fast-time samples the chain reads (rsp_sizes.used_samples)
 * are copied, asynchronously on the plan's upload stream into a plan-owned device ring, so
 * uploads overlap the kernels of earlier batches; with pinned memory (rsp_host_alloc) the copy
 * runs at full PCIe rate.  The host cube must stay unchanged until rsp_drain returns. */
int32_t rsp_enqueue_host(rsp_plan* plan, const void* h_cube, int32_t dtype, int32_t frame_idx);
int32_t rsp_host_alloc(rsp_plan* plan, int64_t bytes, void** h_ptr);   /* pinned host memory */
int32_t rsp_host_free(rsp_plan* plan, void* h_ptr);
int32_t rsp_drain(rsp_plan* plan);
int32_t rsp_results_count(const rsp_plan* plan, int32_t* n_frames, int64_t* n_targets);
int32_t rsp_results_get(const rsp_plan* plan, int32_t i, int32_t* frame_idx, rsp_target* targets,
                        int32_t cap, int32_t* n_targets, int32_t* n_dets);
int32_t rsp_results_clear(rsp_plan* plan);
/* Every queued result as rows of 5 doubles (frame_idx, Range, Velocity, Angle, Power), frames in
 * enqueue order, one NaN row for a frame without targets -- the detection-list payload of the
 * multi-GPU gather, in one call.  *n_rows = rows needed (rows == NULL: a size query);
 * RSP_ERR_OVERFLOW if more than cap. */
int32_t rsp_results_rows(const rsp_plan* plan, double* rows, int64_t cap, int64_t* n_rows);

/* ---- multi-GPU frame batch in one process (BASELINE config #3 for a MEX / loadlibrary host) ----
 * The reference's drivers loop over independent frames (main_simulate_echoes_with_array_v8.m:
 * 164-190, fsf:13 per frame).  Frames j = 0 .. n_frames-1 (targets[j], n_targets[j] targets,
 * frame_idx[j]) are split into contiguous shares over the plans -- plan i, typically one per
 * device, takes [i n / n_plans, (i+1) n / n_plans) -- each driven by its own host thread: S4/S4.1
 * synthesis into the plan's device ring, then the throughput queue.  The final targets of frame j
 * are gathered into out[j * cap ...], n_out[j] entries (the detection-list gather, in process
 * memory).  The plans must have no queued frames or uncleared results.  Synchronous. */
int32_t rsp_process_targets_multi(rsp_plan* const* plans, int32_t n_plans, const rsp_target_in* const* targets,
                                  const int32_t* n_targets, const int32_t* frame_idx, int32_t n_frames,
                                  uint64_t seed, double p_noise, rsp_target* out, int32_t cap, int32_t* n_out);

/* Stage-2 path (process_stage2_mtd.m:1): already-beamformed fast-time data
 * iq_data [P x N x B] (PNC layout with B beams) -> PC_results and MTD_results,
 * both complex [P x G x B] column-major (either may be NULL).  The reference's
 * fun_MTD_produce is un-vendored; this backs it with fsf S6 + S7. */
int32_t rsp_process_stage2(rsp_plan* plan, const void* iq_beams, int32_t dtype,
                           double* mtd_out, double* pc_out);
/* Gated stage-2 input, as the v2 `.mat` frames store it (main_simulate_echoes_with_array_v2.m:
 * 256-267): iq_gated [P x n_gated x B] holds, for segment k = narrow, medium, long, the PRT
 * columns cols[2k] .. cols[2k+1] (1-based, inclusive) side by side.  They are put back at
 * their PRT positions (zeros elsewhere) and processed like rsp_process_stage2.
 * cols = NULL: the reference gating 83:310, 311:1033, 1034:3486 (n_gated = 3404). */
int32_t rsp_process_stage2_gated(rsp_plan* plan, const void* iq_gated, int32_t dtype, int32_t n_gated,
                                 const int32_t* cols, double* mtd_out, double* pc_out);

/* ---- measurement ----
 * Time each device stage `iters` times on the plan's stream with HIP events.  Each launch
 * batches nf = min(n_cubes, frames_per_launch) frames taken from the device-resident
 * cubes d_cubes[] (plan precision); launch j takes cubes (j nf + f) mod n_cubes, f < nf.  ms_out[i] = average ms per launch of stage i,
 * bytes_out[i] = algorithmic HBM bytes per launch (nf frames), *frames_out = nf.
 * Stage names via rsp_stage_name. */
int32_t rsp_profile_stages(rsp_plan* plan, const void* const* d_cubes, int32_t n_cubes, int32_t iters,
                           float* ms_out, int64_t* bytes_out, int32_t cap, int32_t* frames_out);
/* rsp_profile_stages with K2 writing every frame's complex RD map (d_rdms[f], f < nf, as
 * rsp_enqueue_device_rdm); bytes_out[1] then includes the map.  d_rdms = NULL: rsp_profile_stages.
 * d_rdms must hold nf = min(n_cubes, frames_per_launch) non-null maps (a null one is refused with
 * RSP_ERR_INVALID; the array's length cannot be checked here, so the caller sizes it).  A plan with
 * RSP_PLAN_MONOPULSE_COMPLEX writes the map into its own lane buffer on every launch, so its
 * bytes_out[1] includes the map whether or not d_rdms is given. */
int32_t rsp_profile_stages_rdm(rsp_plan* plan, const void* const* d_cubes, int32_t n_cubes, void* const* d_rdms,
                               int32_t iters, float* ms_out, int64_t* bytes_out, int32_t cap, int32_t* frames_out);
const char* rsp_stage_name(int32_t stage);

/* The box's streaming-copy bandwidth (SURVEY 8(d) "measured stream-copy peak"): a 16-B-per-lane
 * non-temporal copy kernel over two device buffers of `bytes` each, `iters` timed launches;
 * *gbps = 2 * bytes / average launch time (read + write).  Measurement only; no plan needed. */
int32_t rsp_hbm_copy_probe(int32_t device, int64_t bytes, int32_t iters, double* gbps);

/* Live stage timing of the throughput queue (rsp_enqueue_device): with timing on, every batch
 * records HIP events around K1, K2 and K3 on the stream the kernels run on, and harvest adds the
 * elapsed times.  rsp_set_stage_timing resets the sums.  rsp_stage_times: ms_sum[i] = total ms
 * of stage i over *launches batched launches holding *frames frames. */
int32_t rsp_set_stage_timing(rsp_plan* plan, int32_t on);
int32_t rsp_stage_times(const rsp_plan* plan, double* ms_sum, int32_t cap, int64_t* launches, int64_t* frames);

/* Host-only S10 + S11 (fun_cluster_stage1_10 / fun_cluster_stage2_11, fsf:302-407) on a
 * detection list (any order; sorted into the reference's find() order first).  No GPU. */
int32_t rsp_cluster_detections(const rsp_detection* dets, int32_t n, const rsp_cluster_params* cluster,
                               rsp_target* out, int32_t cap, int32_t* n_out);

/* ---- inter-frame track association (host only, no GPU) ----
 * main_simulate_echoes_with_array_v8_3.m:253-352: cumulative_final_log (final_targets of every
 * frame with iFrame and iAntAngle injected, :236-244) -> final_tracks_log.  Points are linked
 * when |dRange| <= Gate_R, |dVelocity| <= Gate_V, |d iAntAngle| <= Gate_Az, |dAngle| <= Gate_El
 * and |d iFrame| <= Max_Frame_Gap (config.inter_frame_cluster, v8_3:57-65); clusters are the
 * reference BFS's (connected components, numbered by first member).  Per cluster: the first
 * max-Power member gives Range / Velocity / Angle / Power, Azimuth is the power-weighted mean
 * of iAntAngle, FirstFrame / LastFrame / NumPoints over the members. */
typedef struct rsp_track_point {
    double Range, Velocity, Angle, Power;   /* one final_targets entry (fsf:393-406)     */
    double iAntAngle;                       /* servo azimuth of its frame (v8_3:238)     */
    int32_t iFrame, reserved;               /* frame index (v8_3:237)                    */
} rsp_track_point;

typedef struct rsp_inter_frame_params {
    double Gate_R, Gate_V, Gate_Az, Gate_El;
    int32_t Max_Frame_Gap, reserved;
} rsp_inter_frame_params;

typedef struct rsp_track {   /* one final_tracks_log entry (v8_3:318-335) */
    double Range, Velocity, Angle, Azimuth, Power;
    int32_t FirstFrame, LastFrame, NumPoints, reserved;
} rsp_track;

int32_t rsp_inter_frame_cluster(const rsp_track_point* log, int32_t n, const rsp_inter_frame_params* gates,
                                rsp_track* out, int32_t cap, int32_t* n_out);

/* Device memory helpers (so hosts without a GPU runtime binding can stage cubes). */
int32_t rsp_device_alloc(rsp_plan* plan, int64_t bytes, void** d_ptr);
int32_t rsp_device_free(rsp_plan* plan, void* d_ptr);
int32_t rsp_device_upload(rsp_plan* plan, void* d_dst, const void* h_src, int64_t bytes);
int32_t rsp_device_download(rsp_plan* plan, void* h_dst, const void* d_src, int64_t bytes);
int32_t rsp_device_sync(rsp_plan* plan);

/* ---- MAT-file frame I/O (host only, no GPU) ----
 * The reference moves frames as `frame_sim_array_%d.mat` written by MATLAB's default
 * `save` (-v7: Level-5 format, zlib-compressed elements):
 * main_simulate_echoes_with_array.m:226-229 (`raw_iq_data`),
 * main_simulate_echoes_with_array_v2.m:256-289 (`raw_iq_data_noise_sample`, `servo_angle`),
 * read back by `load` in debug_simulated_data_processing_v3.m:17-22 and
 * main_test_with_simulated_data.m:195,208,215.  These functions replace that MATLAB
 * `save`/`load` pair for hosts without MATLAB.  Level-5 files of either byte order,
 * compressed or not, are read; v7.3 (HDF5) returns RSP_ERR_UNSUPPORTED. */
#define RSP_MAT_MAXDIMS 8
typedef enum rsp_mat_class {    /* MATLAB mxClassID values */
    RSP_MAT_CHAR = 4, RSP_MAT_DOUBLE = 6, RSP_MAT_SINGLE = 7, RSP_MAT_INT8 = 8, RSP_MAT_UINT8 = 9,
    RSP_MAT_INT16 = 10, RSP_MAT_UINT16 = 11, RSP_MAT_INT32 = 12, RSP_MAT_UINT32 = 13,
    RSP_MAT_INT64 = 14, RSP_MAT_UINT64 = 15
} rsp_mat_class;
typedef enum rsp_mat_out {
    RSP_MAT_OUT_F64 = 1,   /* numeric -> double; complex interleaved (mxGetComplexDoubles) */
    RSP_MAT_OUT_F32 = 2,   /* numeric -> float;  complex interleaved                       */
    RSP_MAT_OUT_CHAR = 3   /* char array -> NUL-terminated UTF-8                           */
} rsp_mat_out;

/* One variable of a MAT file as `whos -file` lists it. */
typedef struct rsp_mat_var {
    char name[64];
    int32_t cls;           /* rsp_mat_class (1 cell, 2 struct, 5 sparse, ... listed, not read) */
    int32_t is_complex;
    int32_t ndims;
    int32_t reserved;
    int64_t dims[RSP_MAT_MAXDIMS];
    int64_t numel;
} rsp_mat_var;

/* A variable to write: column-major data, complex interleaved (re, im); cls is
 * RSP_MAT_DOUBLE (data = double*), RSP_MAT_SINGLE (float*) or RSP_MAT_CHAR (bytes). */
typedef struct rsp_mat_wvar {
    const char* name;
    int32_t cls;
    int32_t is_complex;
    int32_t ndims;
    const int64_t* dims;
    const void* data;
} rsp_mat_wvar;

/* List up to `cap` variables (*n_vars = how many the file holds). */
int32_t rsp_mat_list(const char* path, rsp_mat_var* vars, int32_t cap, int32_t* n_vars);
/* Read variable `name` into `out` (cap = entries of out; a complex value counts 2). */
int32_t rsp_mat_read(const char* path, const char* name, int32_t dtype, void* out, int64_t cap);
/* Write a MAT file (Level 5; compress != 0 -> zlib elements like MATLAB -v7). */
int32_t rsp_mat_write(const char* path, const rsp_mat_wvar* vars, int32_t n, int32_t compress);
/* load(frame_sim_array_%d.mat): the [P x N x C] cube (raw_iq_data_noise_sample, else
 * raw_iq_data) into `cube` as dtype RSP_C64/RSP_C128 (NULL: only dims_out), and
 * servo_angle (may be NULL; *n_angle = its length, 0 if absent).  One pass over the file. */
int32_t rsp_mat_load_frame(const char* path, int32_t dtype, void* cube, int64_t cap_elems, int32_t dims_out[3],
                           double* servo_angle, int32_t angle_cap, int32_t* n_angle);
/* save(frame_sim_array_%d.mat, ...): generation 1 -> `raw_iq_data`, 2 ->
 * `raw_iq_data_noise_sample`; complex double cube [P x N x C] interleaved; servo_angle
 * 1 x n_angle (omitted if NULL or n_angle == 0). */
int32_t rsp_mat_save_frame(const char* path, const double* cube, int32_t P, int32_t N, int32_t C,
                           const double* servo_angle, int32_t n_angle, int32_t generation, int32_t compress);

/* ---- MUSIC direction finding (BASELINE config #5) ----
 * MUSIC_1D.m:21-48 and run_music_algorithm.m:22-69: per instance X [N x K] (complex,
 * column-major, instances stacked as [N x K x I]):
 *   R = X*X'/K (MUSIC_1D.m:28); [EV, D] = eig(R), sort 'descend' (:29-32);
 *   Q_n = EV(:, M+1:N) (:33); P = 1./sum(abs(Q_n'*S1).^2) over the scan grid (:35-37);
 *   P_dB = 10*log10(P/max(P)) (:39-41); findpeaks(P_dB), the M largest (:43-47).
 * The reference scripts have no function signature; these entry points take the scripts'
 * variables (N, K, M, d/lambda, phi_list) as the plan and X as the data.  Arithmetic: complex
 * double by default, like MATLAB (f64 MFMA covariance, Householder + multisection + inverse
 * iteration in double); complex single on request (precision = RSP_C64).  Outputs are double
 * either way.  Tolerances vs the complex128 oracle: tests/test_music.py. */
typedef struct rsp_music_config {
    int32_t channel_num;      /* N, 2..64 (MUSIC_1D.m:10; BASELINE #5: 64)                 */
    int32_t num_snapshots;    /* K (MUSIC_1D.m:18; BASELINE #5: 1024)                      */
    int32_t num_sources;      /* M = signal subspace dimension, 1..min(8, N-1) (:15)       */
    int32_t n_scan;           /* scan grid length, 3..4096 (MUSIC_1D.m:35: 200)             */
    double d_over_lambda;     /* element spacing / wavelength (MUSIC_1D.m:11: 0.5)         */
    const double* scan_rad;   /* phi_list in radians, n_scan entries (borrowed for create) */
    int32_t max_batch;        /* instances per call (device buffers sized for it)          */
    int32_t precision;        /* RSP_C128 (complex double, MATLAB's; default) or RSP_C64:
                                 the device snapshots, covariance and eigensolver            */
} rsp_music_config;

/* Synthetic signal model of MUSIC_1D.m:14-24 / run_music_algorithm.m:14-39; MATLAB randn is
 * replaced by the Philox streams documented in oracle/music.py. */
typedef struct rsp_music_scene {
    int32_t n_src;            /* sources, 1..8                                              */
    int32_t complex_sources;  /* 0: Alpha = randn(M,K) (MUSIC_1D.m:22); 1: (randn+1j*randn)/sqrt(2)
                                 (run_music_algorithm.m:30-32); both scaled by amplitudes[m] */
    int32_t snr_measured;     /* 1: awgn(X, SNR, 'measured') (MUSIC_1D.m:24);
                                 0: noise power 1/10^(SNR/10) (run_music_algorithm.m:35)    */
    int32_t reserved;
    double snr_db;
    double angles_rad[8];     /* phi (MUSIC_1D.m:14)                                        */
    double amplitudes[8];     /* source_amplitudes (run_music_algorithm.m:15); 1 for MUSIC_1D */
} rsp_music_scene;

/* Caller-owned outputs for n_inst instances; any pointer may be NULL (not produced). */
typedef struct rsp_music_out {
    double* spectrum_db;      /* [n_scan x I] P_MUSIC_dB (MUSIC_1D.m:41)                      */
    double* eigenvalues;      /* [N x I] descending (MUSIC_1D.m:30-31); when NULL, complex double
                                 (M <= 4) first finds only the signal subspace (the block-power
                                 fast path with a proven 1e-12 subspace bound,
                                 rsp_music_fast_count); a peaks-only call keeps it whenever the
                                 bound is proven, a call that reads spectrum_db only where the
                                 bound also holds P_dB to 1e-8 dB; otherwise (and M > 4) the full
                                 eigensolver finds the M signal eigenvalues the spectrum needs */
    int32_t* peak_idx;        /* [M x I] 1-based scan indices of the M largest peaks (:43-47), 0 = none */
    int32_t* n_peaks;         /* [I] number of findpeaks peaks                                 */
    double* covariance;       /* complex [N x N x I] R (MUSIC_1D.m:28), column-major           */
} rsp_music_out;

typedef struct rsp_music_plan rsp_music_plan;

int32_t rsp_music_create(const rsp_music_config* cfg, int32_t device, rsp_music_plan** out);
int32_t rsp_music_destroy(rsp_music_plan* plan);
/* Host snapshots X [N x K x n_inst] (RSP_C64 or RSP_C128), synchronous. */
int32_t rsp_music_process(rsp_music_plan* plan, const void* X, int32_t dtype, int32_t n_inst, rsp_music_out* out);
/* Device-resident snapshots in the plan's precision ([N x K x n_inst], complex double or single);
 * results copied to `out` (NULL: results stay on the device). */
int32_t rsp_music_process_device(rsp_music_plan* plan, const void* d_X, int32_t n_inst, rsp_music_out* out);
/* Synthesise n_inst instances (instance ids inst0..) into device memory d_X [N x K x n_inst]. */
int32_t rsp_music_synthesize_device(rsp_music_plan* plan, const rsp_music_scene* scene, int32_t n_inst,
                                    int32_t inst0, uint64_t seed, void* d_X);
/* HIP-event timing of the two device stages (ms_out[0] covariance, ms_out[1] eig + spectrum)
 * averaged over `iters` launches on the plan's stream, in the peaks-only form of a call (the
 * eigenvalues not requested: complex double then finds only the M signal eigenvalues). */
int32_t rsp_music_profile(rsp_music_plan* plan, const void* d_X, int32_t n_inst, int32_t iters, float* ms_out);
/* The same timing for the form of call `what` names: RSP_MUSIC_PEAKS (= rsp_music_profile: only
 * peak_idx / n_peaks read; the block-power fast path may stand in for the eigensolver),
 * RSP_MUSIC_SPECTRUM (spectrum_db read too: the fast path only where it bounds P_dB to 1e-8 dB,
 * else the full eigensolver for the M signal eigenvalues) or
 * RSP_MUSIC_EIGENVALUES (eigenvalues read: the full eigensolver, all N eigenvalues -- the
 * 3-output rsp_mex('music') call and music_1d_calllib.m, MUSIC_1D.m:29-33). */
#define RSP_MUSIC_PEAKS 0
#define RSP_MUSIC_SPECTRUM 1
#define RSP_MUSIC_EIGENVALUES 2
int32_t rsp_music_profile_ex(rsp_music_plan* plan, const void* d_X, int32_t n_inst, int32_t iters, int32_t what,
                             float* ms_out);
/* Instances of the last call whose signal subspace came from the block-power fast path (complex
 * double, calls that do not read the eigenvalues, M <= 4: the iteration converged with a proven
 * 1e-12 subspace bound -- and, when spectrum_db is read, that bound holds P_dB to 1e-8 dB;
 * rsp_music.hip me_fast_subspace); the others ran the full tridiagonal eigensolver.  Diagnostic. */
int32_t rsp_music_fast_count(rsp_music_plan* plan, int32_t* n_fast);
int32_t rsp_music_device_alloc(rsp_music_plan* plan, int64_t bytes, void** d_ptr);
int32_t rsp_music_device_free(rsp_music_plan* plan, void* d_ptr);
int32_t rsp_music_device_download(rsp_music_plan* plan, void* h_dst, const void* d_src, int64_t bytes);

#ifdef __cplusplus
}
#endif
#endif /* RSP_H */
