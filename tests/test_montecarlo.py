"""Monte-Carlo angle accuracy -- the reference's only accuracy "test" (main_plot_snr_vs_angle_error.m).

The script (:15-18, :21-29, :62-79) runs the reference frame (16 channels, 13 beams, 5819 x 332,
GOCA 5/10/8) with one target at 10 km, 20 m/s, 10 deg elevation for SNR = -10:2:30 dB, 100
trials each under parfor with fresh MATLAB randn noise (:167-211), records final_targets(1).Angle
- 10 of every trial with a detection (:270-278), and plots std (N-1, omitnan) and Pd per SNR
(:283-284) against the curve |k| sqrt(2) / sqrt(SNR) with k = k_slopes_LUT(5) (:305-309).

Here every trial is rsp_process_targets on the device (complex double): S4 synthesis + S4.1
Philox noise with seed 20250101 + 1000 * i_snr + trial (MATLAB randn is irreproducible), then
S5-S11.  test_snr_vs_angle_error checks the per-frame kernel's estimator -- S9's AMPLITUDE
monopulse on the integer cell, (|A| - |B|) / (|A| + |B| + eps) (fsf:280-290);
test_snr_vs_angle_error_script_estimator runs the script's own inline copy of S9, which uses the
complex ratio real((A - B) / (A + B + eps)) (main_plot_snr_vs_angle_error.m:455-462), through the
plan option monopulse='complex' on a shorter sweep.

Checks:
  * oracle on the same seeds: at -4, 4, 12 and 24 dB the first 8 trials' noisy cubes (downloaded
    from the device) go through oracle.chain in 8 worker processes; every trial's final targets
    must equal the device's (complex double tolerances of test_gpu_parity.py), and the oracle's
    8-seed angle-error std and mean must lie inside the central 99.9 % of the std and mean of
    random 8-trial subsets of the device's 100 trials (a distribution-free bound: the errors are
    heavy-tailed, set by cluster merges, so a Gaussian F test does not apply -- it failed on
    the MI355X at one SNR where one of the first 8 trials is an outlier);
  * Pd = 1 from 0 dB up and never decreases by more than 0.1 between SNR steps; the first final
    target is the true target (|range error| < 15 m) in every detected trial from 0 dB up;
  * the angle-error std stays below the script's curve |k| sqrt(2)/sqrt(SNR) wherever Pd >= 0.9.
    The curve is per-sample: the 16-channel DBF, the 200/700-tap pulse compression and the
    332-pulse MTD put the measured error 1-3 orders of magnitude under it, and what is left is set
    by which cells of which beam pairs cross the threshold and merge in S10/S11 (the
    power-weighted cluster means), not by noise -- so the std is not monotone in SNR (measured on
    the MI355X: 0.03-0.09 deg up to 20 dB, 0.0005-0.0009 deg at 22-28 dB, 0.034 deg at 30 dB
    where an extra pair's cells join).
The per-SNR table is printed (and written to gpurun_out/montecarlo.json when that directory
exists).
"""
import json
import os

import numpy as np
import pytest

from oracle import chain
from rsp import config as C
from rsp.plan import Plan

from _scen import scenario, device_cube

pytestmark = [pytest.mark.gpu, pytest.mark.slow]

SNRS = list(range(-10, 31, 2))          # :15
TRIALS = 100                            # :18
TRUE = dict(Range=10000.0, Velocity=20.0, ElevationAngle=10.0)   # :21-23
K_PAIR5 = C.V8_K_LUT[4]                 # :27-29 (pair 5: beams 9.6 / 16 deg)
SEED0 = 20250101


def _seed(i_snr, trial):
    return SEED0 + 1000 * i_snr + trial


ORACLE_SNRS = (-4, 4, 12, 24)
ORACLE_TRIALS = 8


def _oracle_worker(job):
    """One oracle trial on a downloaded device cube (a worker process: no GPU use)."""
    path, monopulse = job
    from threadpoolctl import threadpool_limits
    from _scen import scenario as sc_
    from oracle import chain as ch
    s = sc_('reference')
    cube = np.load(path)
    with threadpool_limits(2):   # 8 workers x 2 BLAS threads: the box's 16-core share
        return ch.process_cube(cube, s['cfg'], s['cfar'], s['clus'], s['pre_o'], monopulse=monopulse)


def _oracle_trials(plan, todo, tmpdir, workers=8, monopulse='amplitude'):
    """{(snr, trial): oracle final targets} on the device's own noisy cubes, `workers` at a time."""
    import multiprocessing as mp
    out = {}
    ctx = mp.get_context('spawn')
    with ctx.Pool(workers) as pool:
        for k in range(0, len(todo), workers):
            chunk = todo[k:k + workers]
            paths = []
            for snr, t in chunk:
                cube = device_cube(plan, [dict(TRUE, SNR_dB=float(snr))], frame_idx=1, seed=_seed(SNRS.index(snr), t))
                pth = os.path.join(tmpdir, 'cube_%d_%d.npy' % (snr + 100, t))
                np.save(pth, cube)
                paths.append(pth)
            for key, fo, pth in zip(chunk, pool.map(_oracle_worker, [(q, monopulse) for q in paths]), paths):
                out[key] = fo
                os.remove(pth)
    return out


def test_snr_vs_angle_error(tmp_path):
    s = scenario('reference')
    plan = Plan(s['cfg'], s['cfar'], s['clus'], s['pre_p'])
    table = []
    dev = {}
    dev_errs = {}
    try:
        for i, snr in enumerate(SNRS):
            tg = [dict(TRUE, SNR_dB=float(snr))]
            errs, rng_errs, n_det = [], [], 0
            for t in range(TRIALS):
                fin = plan.process_targets(tg, frame_idx=1, seed=_seed(i, t))['final_targets']
                if snr in ORACLE_SNRS and t < ORACLE_TRIALS:
                    dev[(snr, t)] = fin
                if fin:
                    n_det += 1
                    errs.append(fin[0]['Angle'] - TRUE['ElevationAngle'])     # :274-275
                    rng_errs.append(fin[0]['Range'] - TRUE['Range'])
            dev_errs[snr] = errs
            std = float(np.std(errs, ddof=1)) if len(errs) > 1 else float('nan')   # std(..., 'omitnan')
            theory = abs(K_PAIR5) * np.sqrt(2) / np.sqrt(10 ** (snr / 10))      # :306-308
            table.append(dict(snr_db=snr, pd=n_det / TRIALS, angle_err_std=std, theory=theory,
                              angle_err_mean=float(np.mean(errs)) if errs else float('nan'),
                              max_abs_range_err=float(np.max(np.abs(rng_errs))) if rng_errs else float('nan'),
                              n_detected=len(errs)))
        # the oracle on the same seeds (the device's own cubes), per trial and per SNR
        orc = _oracle_trials(plan, sorted(dev), str(tmp_path))
        for key, fin in sorted(dev.items()):
            fo = orc[key]
            assert len(fo) == len(fin), key
            for a, b in zip(fo, fin):
                for f in ('Range', 'Velocity', 'Angle', 'Power'):
                    assert b[f] == pytest.approx(a[f], rel=1e-9, abs=1e-9), (key, f)
        for r in table:
            if r['snr_db'] not in ORACLE_SNRS:
                continue
            e = [orc[(r['snr_db'], t)][0]['Angle'] - TRUE['ElevationAngle'] for t in range(ORACLE_TRIALS)
                 if orc[(r['snr_db'], t)]]
            so, mo, no = float(np.std(e, ddof=1)), float(np.mean(e)), len(e)
            r.update(oracle_std=so, oracle_mean=mo, oracle_n=no)
            # distribution-free bound (the errors are heavy-tailed: cluster merges, not Gaussian
            # noise): the oracle's std / mean over its no seeds must lie inside the central
            # 99.9 % of the std / mean of random no-trial subsets of the device's trials
            d = np.asarray(dev_errs[r['snr_db']])
            rng = np.random.default_rng(r['snr_db'] + 1000)
            sub = np.stack([rng.choice(d, no, replace=False) for _ in range(20000)])
            sd_q = np.quantile(np.std(sub, axis=1, ddof=1), [0.0005, 0.9995])
            mu_q = np.quantile(np.mean(sub, axis=1), [0.0005, 0.9995])
            r.update(subset_std_q=[float(x) for x in sd_q], subset_mean_q=[float(x) for x in mu_q])
            assert sd_q[0] <= so <= sd_q[1], r
            assert mu_q[0] <= mo <= mu_q[1], r
    finally:
        plan.close()
    print()
    for r in table:
        print('SNR %+3d dB  Pd %.2f  std %.4f deg  (curve %.4f)  mean %+.4f  max|dR| %.2f m%s' % (
            r['snr_db'], r['pd'], r['angle_err_std'], r['theory'], r['angle_err_mean'], r['max_abs_range_err'],
            '  oracle (%d trials) std %.4f mean %+.4f' % (r['oracle_n'], r['oracle_std'], r['oracle_mean'])
            if 'oracle_std' in r else ''))
    out = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'gpurun_out')
    if os.path.isdir(out):
        json.dump(table, open(os.path.join(out, 'montecarlo.json'), 'w'), indent=1)
    by = {r['snr_db']: r for r in table}
    for r in table:
        if r['snr_db'] >= 0:
            assert r['pd'] == 1.0, r
            assert r['max_abs_range_err'] < 15.0, r
        if r['pd'] >= 0.9:
            assert r['angle_err_std'] < r['theory'], r
    for a, b in zip(table, table[1:]):
        assert b['pd'] >= a['pd'] - 0.1, (a, b)
    assert by[30]['pd'] == 1.0


def test_snr_vs_angle_error_script_estimator(tmp_path):
    """The script's own estimator: its inline S9 takes the angle from the complex ratio
    real((S_A - S_B) / (S_A + S_B + eps)) (main_plot_snr_vs_angle_error.m:455-462), which the plan
    runs with monopulse='complex' (RSP_PLAN_MONOPULSE_COMPLEX).  A shorter sweep than the script's
    (4 SNRs x 32 trials): every one of the first 4 trials per SNR equals the oracle's complex-ratio
    chain on the same cube, Pd = 1 from 0 dB up, and the angle-error std stays below the script's
    curve |k| sqrt(2) / sqrt(SNR) wherever Pd >= 0.9."""
    s = scenario('reference')
    plan = Plan(s['cfg'], s['cfar'], s['clus'], s['pre_p'], monopulse='complex')
    snrs, trials, n_orc = (-4, 4, 12, 24), 32, 4
    table, dev = [], {}
    try:
        for snr in snrs:
            i = SNRS.index(snr)
            tg = [dict(TRUE, SNR_dB=float(snr))]
            errs, n_det = [], 0
            for t in range(trials):
                fin = plan.process_targets(tg, frame_idx=1, seed=_seed(i, t))['final_targets']
                if t < n_orc:
                    dev[(snr, t)] = fin
                if fin:
                    n_det += 1
                    errs.append(fin[0]['Angle'] - TRUE['ElevationAngle'])
            table.append(dict(snr_db=snr, pd=n_det / trials, n_detected=len(errs),
                              angle_err_std=float(np.std(errs, ddof=1)) if len(errs) > 1 else float('nan'),
                              angle_err_mean=float(np.mean(errs)) if errs else float('nan'),
                              theory=abs(K_PAIR5) * np.sqrt(2) / np.sqrt(10 ** (snr / 10))))
        orc = _oracle_trials(plan, sorted(dev), str(tmp_path), workers=8, monopulse='complex')
        for key, fin in sorted(dev.items()):
            fo = orc[key]
            assert len(fo) == len(fin), key
            for a, b in zip(fo, fin):
                for f in ('Range', 'Velocity', 'Angle', 'Power'):
                    assert b[f] == pytest.approx(a[f], rel=1e-9, abs=1e-9), (key, f)
    finally:
        plan.close()
    print()
    for r in table:
        print('complex ratio: SNR %+3d dB  Pd %.2f  std %.4f deg  (curve %.4f)  mean %+.4f' % (
            r['snr_db'], r['pd'], r['angle_err_std'], r['theory'], r['angle_err_mean']))
    out = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'gpurun_out')
    if os.path.isdir(out):
        json.dump(table, open(os.path.join(out, 'montecarlo_complex.json'), 'w'), indent=1)
    for r in table:
        if r['snr_db'] >= 0:
            assert r['pd'] == 1.0, r
        if r['pd'] >= 0.9:
            assert r['angle_err_std'] < r['theory'], r
