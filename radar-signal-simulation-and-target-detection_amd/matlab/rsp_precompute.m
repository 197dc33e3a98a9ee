function pre = rsp_precompute(config)
%RSP_PRECOMPUTE  precomputed_data of main_simulate_echoes_with_array_v8.m:79-135 from config alone:
%   waveform (v8:80-98), matched filters (v8:101-123), segment geometry (v8:126-132), MTD window
%   and axes (v8:135-142).  The DBF weights, beam angles and K-LUT (v8:138-155) are not used by
%   the stage-2 path and are zero here.  Same computation as rsp/precompute.py (tested there).
sc = config.Sig_Config;
fs = sc.fs; N = sc.point_PRT; P = sc.prtNum; B = sc.beam_num; C = sc.channel_num;
tau1 = sc.tao(1); tau2 = sc.tao(2); tau3 = sc.tao(3);
gap1 = sc.gap_duration(1); gap2 = sc.gap_duration(2);
n1 = round(tau1 * fs); n2 = round(tau2 * fs); n3 = round(tau3 * fs);
t2 = linspace(-tau2/2, tau2/2, n2);
t3 = linspace(-tau3/2, tau3/2, n3);
pulse2 = exp(1j*2*pi*(0.5*(-sc.B/tau2)*(t2.^2)));
pulse3 = exp(1j*2*pi*(0.5*(sc.B/tau3)*(t3.^2)));
tx = complex(zeros(1, N));
tx(1:n1) = 1;
o1 = round((tau1 + gap1) * fs);
tx(o1+1 : o1+n2) = pulse2;
o2 = o1 + round((tau2 + gap2) * fs);
tx(o2+1 : o2+n3) = pulse3;
pre.tx_pulse = tx;
pre.P_signal_unscaled = mean(abs(tx(tx ~= 0)).^2);
fir = [794,1403,2143,2672,2591,1711,-58,-2351,-4592,-5855,-5338,-2389,3005,10341,18410,25779,30907,32768, ...
       30907,25779,18410,10341,3005,-2389,-5338,-5855,-4592,-2351,-58,1711,2591,2672,2143,1403,794];
pre.MF_narrow = 6 * fir / max(fir);
pre.fir_delay = round(mean(grpdelay(pre.MF_narrow)));
MF_medium_win = fliplr(conj(pulse2 .* kaiser(n2, 4.5)'));
MF_long_win = fliplr(conj(pulse3 .* kaiser(n3, 4.5)'));
ssm = n1 + gap1 * fs + n2 + 1;
ssl = n1 + gap1 * fs + n2 + gap2 * fs + n3 + 1;
pre.N_fft_med = 2^nextpow2(N - ssm + 1 + n2 - 1);
pre.N_fft_long = 2^nextpow2(N - ssl + 1 + n3 - 1);
pre.MF_medium_fft = fft(MF_medium_win, pre.N_fft_med);
pre.MF_long_fft = fft(MF_long_win, pre.N_fft_long);
seg = sc.point_prt_segments;
pre.N_gate_narrow = seg(1); pre.N_gate_medium = seg(2); pre.N_gate_long = seg(3);
pre.N_total_gate = sum(seg);
pre.seg_start_narrow = n1 + 1; pre.seg_start_medium = ssm; pre.seg_start_long = ssl;
pre.MTD_win = kaiser(P, 4.5);
v_max = sc.wavelength / (2 * sc.prt);
pre.velocity_axis = linspace(-v_max/2, v_max/2, P);
pre.range_axis = (0:pre.N_total_gate-1) * (sc.c / (2 * fs));
pre.deltaR = sc.c / fs / 2;
pre.deltaV = v_max / P;
pre.beam_angles_deg = zeros(1, B);
pre.k_slopes_LUT = zeros(1, max(B - 1, 1));
pre.DBF_coeffs_data_C = complex(zeros(B, C));
end
