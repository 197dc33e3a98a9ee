function [phi_e, P_MUSIC_dB, EVA, R] = music_1d_gpu(X1, M, phi_list, d_over_lambda, opts)
% MI355X drop-in for the MUSIC section of MUSIC_1D.m (:26-48) through the MEX gateway rsp_mex.c.
% X1 [N x K] complex snapshots (or a batch [N x K x I]), M sources, phi_list the scan grid in rad
% (MUSIC_1D.m:35), d_over_lambda = d / lambda (MUSIC_1D.m:11).  phi_e [M x I] in degrees
% (MUSIC_1D.m:47), P_MUSIC_dB [numel(phi_list) x I] (:41), EVA [N x I] descending (:30-31),
% R [N x N x I] (:28).  opts (optional): device, precision ('double' default | 'single').
if nargin < 5
    opts = struct();
end
[phi_e, P_MUSIC_dB, EVA, R] = rsp_mex('music', X1, M, phi_list, d_over_lambda, opts);
end
