function [MTD_results, PC_results] = process_stage2_mtd(iq_data, angle, config)
%PROCESS_STAGE2_MTD  MI355X drop-in for process_stage2_mtd.m:1 (librsp.so via rsp_mex).
%   iq_data: beamformed fast-time data [P x n x B] (debug_simulated_data_processing_v3.m:146-152),
%   n = point_PRT (the full PRT) or the 3404 columns of the v2 .mat frames
%   (main_simulate_echoes_with_array_v2.m:256-267: PRT columns 83:310, 311:1033, 1034:3486; set
%   config.rsp_gate_cols = [first last; first last; first last] for another gating).  angle is
%   unused, as in the reference.  Returns complex [P x N_total_gate x B] arrays
%   (process_stage2_mtd.m:29-30).  The reference's fun_MTD_produce is not part of the reference
%   repository; this runs the per-frame chain's own pulse compression and MTD (fsf:99-136) with
%   precomputed_data built from config like v8:79-135 (rsp_precompute.m).
persistent pre key
k = config.Sig_Config;
if isempty(pre) || ~isequal(key, k)
    pre = rsp_precompute(config);
    key = k;
end
opts = struct();
if isfield(config, 'rsp_gate_cols'), opts.gate_cols = config.rsp_gate_cols; end
[MTD_results, PC_results] = rsp_mex('stage2', iq_data, config, pre, opts);
end
