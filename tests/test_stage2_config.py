"""The stage-2 path's config normalisation (rsp.config.stage2_config) on the caller's own config,
debug_simulated_data_processing_v3.m:55-106 (process_stage2_mtd is called from :189 with it):
it describes the reference frame's waveform and gating, so the precomputed_data built from it
must equal v8:79-135's for the reference config, field by field.  CPU only."""
import numpy as np

from rsp import config as C
from rsp import _stage2_precompute


def test_debug_v3_config_gives_reference_geometry():
    v3 = C.stage2_config(C.debug_v3_config())
    sc = v3['Sig_Config']
    assert sc['point_PRT'] == 5819 and sc['beam_num'] == 13 and sc['point_prt_segments'] == [228, 723, 2453]
    ref = C.stage2_config(C.named_config('reference')[0])
    a, b = _stage2_precompute(v3), _stage2_precompute(ref)
    for k in ('tx_pulse', 'MF_narrow', 'MF_medium_fft', 'MF_long_fft', 'MTD_win', 'range_axis', 'velocity_axis'):
        np.testing.assert_array_equal(a[k], b[k], err_msg=k)
    for k in ('fir_delay', 'N_fft_med', 'N_fft_long', 'N_gate_narrow', 'N_gate_medium', 'N_gate_long',
              'N_total_gate', 'seg_start_narrow', 'seg_start_medium', 'seg_start_long', 'deltaR', 'deltaV'):
        assert a[k] == b[k], k
    assert a['N_total_gate'] == 3404 and (a['seg_start_medium'], a['seg_start_long']) == (490, 1985)


def test_stage2_config_keeps_v8_configs():
    for name in ('reference', 'x2', 'small'):
        cfg = C.named_config(name)[0]
        out = C.stage2_config(cfg)
        for k in ('prtNum', 'point_PRT', 'channel_num', 'beam_num', 'point_prt_segments', 'gap_duration', 'tao'):
            assert out['Sig_Config'][k] == cfg['Sig_Config'][k], (name, k)
        assert out['Array'] == cfg['Array']


def test_stage2_config_keeps_the_callers_c():
    """A caller-supplied Sig_Config.c is honoured and the wavelength follows it, as in
    matlab/process_stage2_mtd.m (s.c = sc.c; s.wavelength = s.c / s.fc)."""
    cfg = C.debug_v3_config()
    cfg['Sig_Config']['c'] = 3e8
    sc = C.stage2_config(cfg)['Sig_Config']
    assert sc['c'] == 3e8 and sc['wavelength'] == 3e8 / sc['fc']
    assert C.stage2_config(C.debug_v3_config())['Sig_Config']['c'] == C.C_LIGHT
