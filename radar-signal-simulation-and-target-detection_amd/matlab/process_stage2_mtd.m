function [MTD_results, PC_results] = process_stage2_mtd(iq_data, angle, config)
%PROCESS_STAGE2_MTD  MI355X drop-in for process_stage2_mtd.m:1 (librsp.so via rsp_mex).
%   iq_data: beamformed fast-time data [P x n x B] (debug_simulated_data_processing_v3.m:146-152),
%   n = the full PRT or the 3404 columns of the v2 .mat frames
%   (main_simulate_echoes_with_array_v2.m:256-267: PRT columns 83:310, 311:1033, 1034:3486; set
%   config.rsp_gate_cols = [first last; first last; first last] for another gating).  angle is
%   unused, as in the reference.  Returns complex [P x N_total_gate x B] arrays
%   (process_stage2_mtd.m:29-30).  The reference's fun_MTD_produce is not part of the reference
%   repository; this runs the per-frame chain's own pulse compression and MTD (fsf:99-136) with
%   precomputed_data built from config like v8:79-135 (rsp_precompute.m).
%
%   config may be the v8 drivers' form or the caller's own, debug_simulated_data_processing_v3.m:
%   55-106 (point_PRT = 3404 gated samples, point_prt = [3404 228 723 2453], no gap_duration,
%   no Array, config.mtd.beam_num).  stage2_config below turns either into the v8 form: full PRT
%   round(prt*fs) (v8:68), B = config.mtd.beam_num when present (process_stage2_mtd.m:15), gate
%   counts point_prt_segments or else point_prt(2:4), gaps gap_duration or else the reference
%   waveform's (v8:61).  Same rule as rsp/config.py stage2_config (tested there).
persistent pre key
cfg = stage2_config(config);
if isempty(pre) || ~isequal(key, cfg.Sig_Config)
    pre = rsp_precompute(cfg);
    key = cfg.Sig_Config;
end
opts = struct();
if isfield(config, 'rsp_gate_cols'), opts.gate_cols = config.rsp_gate_cols; end
[MTD_results, PC_results] = rsp_mex('stage2', iq_data, cfg, pre, opts);
end

function cfg = stage2_config(config)
sc = config.Sig_Config;
s = struct();
s.c = sc.c; s.fs = sc.fs; s.fc = sc.fc; s.B = sc.B; s.tao = sc.tao;
if isfield(sc, 'prt'), s.prt = sc.prt; else, s.prt = sc.point_PRT / sc.fs; end
s.prtNum = sc.prtNum;
if isfield(sc, 'point_prt_segments')
    s.point_prt_segments = sc.point_prt_segments;
else
    s.point_prt_segments = sc.point_prt(2:4);
end
if isfield(sc, 'gap_duration'), s.gap_duration = sc.gap_duration; else, s.gap_duration = [11.4e-6, 31.8e-6, 153.4e-6]; end
if isfield(config, 'mtd') && isfield(config.mtd, 'beam_num'), s.beam_num = config.mtd.beam_num; else, s.beam_num = sc.beam_num; end
if isfield(sc, 'channel_num'), s.channel_num = sc.channel_num; else, s.channel_num = s.beam_num; end
s.wavelength = s.c / s.fc;
s.point_PRT = round(s.prt * s.fs);
cfg.Sig_Config = s;
if isfield(config, 'Array') && isfield(config.Array, 'element_spacing')
    cfg.Array.element_spacing = config.Array.element_spacing;
else
    cfg.Array.element_spacing = 0.0138;   % not used by stage 2
end
end
