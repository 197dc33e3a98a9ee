function [phi_e, P_MUSIC_dB, EVA] = music_1d_calllib(X1, M, phi_list, d_over_lambda)
% MUSIC_1D.m:26-48 on librsp.so through loadlibrary/calllib (no compiler needed).  The types of
% every libstruct field and libpointer follow include/rsp.h (tests/test_mex_gateway.py checks
% them): rsp_music_config.precision = 2 (RSP_C128, complex double like MATLAB), double outputs.
if ~libisloaded('librsp')
    loadlibrary('librsp', 'rsp.h');
end
[N, K] = size(X1);
nscan = numel(phi_list);
scan = libpointer('doublePtr', double(phi_list(:).'));
cfg = libstruct('rsp_music_config', struct('channel_num', int32(N), 'num_snapshots', int32(K), ...
    'num_sources', int32(M), 'n_scan', int32(nscan), 'd_over_lambda', double(d_over_lambda), ...
    'scan_rad', scan, 'max_batch', int32(1), 'precision', int32(2)));
plan = libpointer('voidPtr');   % a ** argument receives the address of a voidPtr
if calllib('librsp', 'rsp_music_create', cfg, int32(0), plan) ~= 0
    error('radar:rsp', calllib('librsp', 'rsp_last_error'));
end
spec = libpointer('doublePtr', zeros(1, nscan));
eva = libpointer('doublePtr', zeros(1, N));
pk = libpointer('int32Ptr', zeros(1, M, 'int32'));
npk = libpointer('int32Ptr', int32(0));
cov = libpointer('doublePtr');
out = libstruct('rsp_music_out', struct('spectrum_db', spec, 'eigenvalues', eva, 'peak_idx', pk, ...
    'n_peaks', npk, 'covariance', cov));
x = libpointer('doublePtr', reshape([real(X1(:)).'; imag(X1(:)).'], 1, []));   % interleaved complex double
rc = calllib('librsp', 'rsp_music_process', plan, x, int32(2), int32(1), out);
calllib('librsp', 'rsp_music_destroy', plan);
if rc ~= 0
    error('radar:rsp', calllib('librsp', 'rsp_last_error'));
end
P_MUSIC_dB = spec.Value(:);
EVA = eva.Value(:);
idx = pk.Value(pk.Value > 0);
phi_e = phi_list(idx) * 180 / pi;
end
