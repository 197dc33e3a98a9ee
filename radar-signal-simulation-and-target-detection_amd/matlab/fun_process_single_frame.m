function final_targets = fun_process_single_frame(targets, config, cfar_params, cluster_params, precomputed_data, frame_idx)
%FUN_PROCESS_SINGLE_FRAME  MI355X drop-in for fun_process_single_frame.m:13 (librsp.so via rsp_mex).
%   Same signature and result as the reference: final_targets is a 1 x K struct array with
%   Range, Velocity, Angle, Power (fun_process_single_frame.m:393-406).  Put this folder ahead of
%   Simulation/ on the path; the v8 drivers (v8:177, v8_1:195, v8_2:208, v8_3:232) are unchanged.
%   S4 echo synthesis and S4.1 noise run on the GPU: MATLAB randn is replaced by the Philox
%   stream of seed 20250101 and frame_idx.  Arithmetic is complex double, like MATLAB.  The
%   device plan is cached inside rsp_mex and rebuilt whenever any of the input structs changes.
final_targets = rsp_mex('frame', targets, config, cfar_params, cluster_params, precomputed_data, frame_idx);
end
