#!/usr/bin/env python3
"""Throughput bench of the per-frame radar chain on MI355X (BASELINE.json config #2).

Workload: 16-channel x 8-beam x 4096-sample x 128-pulse echo cubes (BASELINE config #2,
``named_config('x2')``), synthetic: the v8_2 five-target scene (v8_2:28-51) evolved per
frame (v8:170-173) plus Philox noise, synthesised ON the device into a ring of distinct
frame cubes (ring > 256 MiB Infinity Cache, so every step reads its cube from HBM).
One step = one batch of ``--fpl`` distinct frames (one launch of each kernel) through
DBF -> MTD -> pulse compression -> GOCA-CFAR -> S9 estimation (device) -> S10/S11
clustering (host); batches rotate over the plan's lanes (3 HIP streams).  Warm-up
always runs at least WARM_MIN = 100 batches (every lane, settled clocks) whatever ``--warmup`` says.
``value`` is frames/s = steps x fpl / time; inside the timed region the frames are
queued with one C call and every frame's final targets come back as packed rows.

Multi-GPU: one process per GPU (torchrun); frames are sharded (each rank processes its
own K frames, weak scaling); the only collective is an RCCL all-gather of the
detection lists at the end (inside the timed region).

Prints ONE JSON line (rank 0).
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(ROOT, 'radar-signal-simulation-and-target-detection_amd')
for _p in (ROOT, PKG):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import numpy as np  # noqa: E402

HBM_PEAK_GBS = 8000.0   # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
NLANES = 3              # streams of the plan's throughput queue (rsp_plan.cpp)
# untimed warm-up floor in batches (~55 ms at x2): a 20-step timed region after 20 warm-up batches ran
# 11.7-11.9 ms, after 60 or 200 batches 11.4 ms on the same box (the GPU's clocks still ramping)
WARM_MIN = 100


def host_cpu():
    """CPU model, nproc, the affinity set and the cgroup CPU quota of this host; `usable` =
    the threads the CPU baseline may run (the affinity set capped by the quota)."""
    model = 'unknown'
    try:
        with open('/proc/cpuinfo') as f:
            for line in f:
                if line.startswith('model name'):
                    model = line.split(':', 1)[1].strip()
                    break
    except OSError:
        pass
    aff = len(os.sched_getaffinity(0))
    quota = None
    try:
        with open('/sys/fs/cgroup/cpu.max') as f:
            q, per = f.read().split()
            if q != 'max':
                quota = int(q) / int(per)
    except (OSError, ValueError):
        pass
    usable = aff if quota is None else max(1, min(aff, int(quota)))
    return {'model': model, 'nproc': os.cpu_count(), 'affinity': aff, 'cgroup_quota': quota, 'usable': usable}


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1,
                    help='GPUs (ranks) of the run: under torchrun it must equal WORLD_SIZE; without it, N > 1 '
                         'spawns N ranks through torch.distributed.run and relays rank 0\'s line')
    ap.add_argument('--steps', type=int, default=500)
    ap.add_argument('--warmup', type=int, default=20)
    ap.add_argument('--config', default='x2')
    ap.add_argument('--precision', default='c128', choices=['c128', 'c64'],
                    help="c128: complex double, the reference's MATLAB arithmetic (default); c64: complex single")
    ap.add_argument('--fpl', type=int, default=8, help='frames per launch (8: fewest tail rounds, measured)')
    ap.add_argument('--ring', type=int, default=8, help='distinct device-resident frame cubes')
    ap.add_argument('--profile-iters', type=int, default=50)
    ap.add_argument('--cpu-frames', type=int, default=0, help='oracle frames for cpu_baseline (0 = auto ~15 s)')
    ap.add_argument('--no-cpu-baseline', action='store_true')
    ap.add_argument('--batch', type=int, default=4096,
                    help='MUSIC instances per launch (--config music5; 4096: 2.30 vs 1.96-2.14 M instances/s at 1024, '
                         'profiles/r05w_music_batch.txt)')
    ap.add_argument('--frames-total', type=int, default=0,
                    help='BASELINE config #3 mode: this many distinct frames (e.g. 512), sharded over the ranks, '
                         'each processed once (the default mode times --steps batches over a ring)')
    ap.add_argument('--e2e', action='store_true',
                    help='end-to-end mode: frames enter as host cubes in pinned memory (rsp_enqueue_host: '
                         'async H2D of the used samples overlapping the kernels), not the headline')
    ap.add_argument('--dist-backend', default='nccl', choices=['nccl', 'gloo'],
                    help='collective backend for N > 1 (nccl = RCCL over xGMI; gloo: CPU tensors, for rehearsing '
                         'several ranks on one GPU together with --same-device)')
    ap.add_argument('--same-device', action='store_true', help='every rank uses GPU 0 (rehearsal only)')
    ap.add_argument('--want-rdm', action='store_true',
                    help='every frame also writes its complex range-Doppler map (rdm_13beam, fsf:131-136) to a '
                         'device buffer of the caller (rsp_enqueue_device_rdm): the rsp_mex(\'cube\') contract; '
                         'a secondary line, not the headline')
    ap.add_argument('--stage-timing', action='store_true',
                    help='HIP events around every kernel in the timed region (diagnostic: overlapped durations)')
    ap.add_argument('--want-eig', action='store_true',
                    help='--config music5: every step also returns all N eigenvalues (the 3-output rsp_mex(\'music\') '
                         'and music_1d_calllib.m form, MUSIC_1D.m:29-33): the full eigensolver, never the '
                         'peaks-only fast path; a secondary line')
    ap.add_argument('--want-spectrum', action='store_true',
                    help='--config music5: every step also returns the pseudo-spectrum P_dB (the 2-output '
                         'rsp_mex(\'music\') form and MUSIC_1D.m\'s plot, :37-41): the fast path only where its '
                         'subspace bound holds P_dB to 1e-8 dB; a secondary line')
    ap.add_argument('--per-call', action='store_true',
                    help='latency mode: --steps synchronous rsp_process_targets calls, one frame each, timed one by '
                         'one like the v8 frame loop\'s tic/toc (v8:162,177,191-194); not the headline')
    return ap.parse_args(argv)


def launch_mode(gpus, env_world, visible, same_device, backend):
    """What `bench.py --gpus N` does: ('run', None) in this process (N = 1, or a torchrun rank whose
    WORLD_SIZE is N), ('spawn', None) to start N ranks, or ('error', message).  Pure: no GPU call;
    `visible` = visible_gpus() (counted without the HIP runtime)."""
    if gpus < 1:
        return 'error', '--gpus must be >= 1, got %d' % gpus
    if env_world is not None:   # a rank started by torchrun / torch.distributed.run
        if env_world != gpus:
            return 'error', '--gpus %d but WORLD_SIZE=%d: launch one rank per GPU with --nproc-per-node %d' % (
                gpus, env_world, gpus)
        return 'run', None
    if gpus == 1:
        return 'run', None
    if same_device:
        if backend == 'nccl':
            return 'error', ('--same-device puts every rank on GPU 0, which RCCL refuses; '
                             'rehearse with --dist-backend gloo')
    elif visible < gpus:
        return 'error', '--gpus %d but only %d GPU(s) visible (rehearse on one GPU with --same-device ' \
                        '--dist-backend gloo)' % (gpus, visible)
    return 'spawn', None


def visible_gpus():
    """GPUs this process could open, counted without HIP (no torch.cuda, no amdsmi, no HIP
    runtime loaded): KFD topology nodes with a non-zero gpu_id whose DRM render node opens
    read-write here (a container or cgroup that hides a GPU makes its node absent or its open
    fail), then filtered by ROCR_VISIBLE_DEVICES / HIP_VISIBLE_DEVICES / CUDA_VISIBLE_DEVICES
    the way the ROCm runtime applies them (a list of ordinals; empty = none)."""
    import glob
    n = 0
    for node in sorted(glob.glob('/sys/class/kfd/kfd/topology/nodes/*')):
        try:
            with open(os.path.join(node, 'gpu_id')) as f:
                if int(f.read().strip() or 0) == 0:
                    continue   # a CPU node
            minor = None
            with open(os.path.join(node, 'properties')) as f:
                for line in f:
                    if line.startswith('drm_render_minor'):
                        minor = int(line.split()[1])
            if minor is None:
                continue
            fd = os.open('/dev/dri/renderD%d' % minor, os.O_RDWR | os.O_CLOEXEC)
            os.close(fd)
            n += 1
        except (OSError, ValueError):
            continue
    for var in ('ROCR_VISIBLE_DEVICES', 'HIP_VISIBLE_DEVICES', 'CUDA_VISIBLE_DEVICES'):
        v = os.environ.get(var)
        if v is not None:
            ids = [s for s in v.split(',') if s.strip() != '']
            n = min(n, len(ids))
    return n


def rank_census(dist, dev):
    """What the process group actually is, for the JSON line: world size and backend as
    torch.distributed reports them, and every rank's device (ordinal, PCI location, UUID)
    gathered to all ranks.  A collective: every rank calls it."""
    import torch
    me = {'rank': dist.get_rank(), 'local_rank': int(os.environ.get('LOCAL_RANK', 0)), 'device': dev,
          'pid': os.getpid()}
    try:
        pr = torch.cuda.get_device_properties(dev)
        me['device_name'] = pr.name
        for k in ('pci_domain_id', 'pci_bus_id', 'pci_device_id'):
            if hasattr(pr, k):
                me[k] = int(getattr(pr, k))
        if hasattr(pr, 'uuid'):
            me['uuid'] = str(pr.uuid)
    except Exception as e:   # the census must not fail the run
        me['device_error'] = repr(e)
    allr = [None] * dist.get_world_size()
    dist.all_gather_object(allr, me)
    devs = {(r.get('pci_domain_id'), r.get('pci_bus_id'), r.get('pci_device_id'), r.get('uuid'), r['device'])
            for r in allr}
    return {'world_size': dist.get_world_size(), 'backend': str(dist.get_backend()),
            'distinct_devices': len(devs), 'ranks': allr}


def validate_args(a):
    """Argument combinations that would report work that is not done: an error message or None."""
    if a.want_rdm and a.e2e:
        return ('--want-rdm with --e2e: the end-to-end queue (rsp_enqueue_host) does not write the '
                'complex RD map, so the line would claim map bytes that were never stored')
    if a.want_rdm and a.config == 'music5':
        return '--want-rdm applies to the radar chain, not --config music5'
    if a.want_eig and a.config != 'music5':
        return '--want-eig applies to --config music5 only'
    if a.want_spectrum and (a.config != 'music5' or a.want_eig):
        return '--want-spectrum applies to --config music5 only, without --want-eig (which returns the spectrum\'s superset)'
    if a.per_call and (a.config == 'music5' or a.e2e or a.want_rdm or a.frames_total or a.gpus != 1):
        return ('--per-call times single synchronous frames of the radar chain on one GPU: it takes none of '
                '--config music5, --e2e, --want-rdm, --frames-total, --gpus N')
    return None


def spawn_ranks(gpus, argv):
    """Start `gpus` ranks of this script with torch.distributed.run (rendezvous on 127.0.0.1) as a
    child process -- this process never touches the GPU -- and relay rank 0's JSON line."""
    import socket
    import subprocess
    sk = socket.socket()
    sk.bind(('127.0.0.1', 0))
    port = sk.getsockname()[1]
    sk.close()
    cmd = [sys.executable, '-m', 'torch.distributed.run', '--nnodes=1', '--nproc-per-node', str(gpus),
           '--master-addr', '127.0.0.1', '--master-port', str(port), os.path.abspath(__file__)] + list(argv)
    r = subprocess.run(cmd, stdout=subprocess.PIPE, text=True)
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith('{')]
    if r.returncode != 0 or not lines:
        sys.stderr.write(r.stdout)
        return r.returncode or 1
    print(lines[-1])
    return 0


def scene(cfg):
    from rsp import config as C
    sc = cfg['Sig_Config']
    G = sum(sc['point_prt_segments'])
    rmax = 0.9 * G * sc['c'] / (2 * sc['fs'])
    return [t for t in C.v8_2_targets() if t['Range'] < rmax]


def cpu_baseline(cfg, cfar, clus, W, ang, k, targets, budget_s=15.0, nframes=0, name='x2'):
    """The oracle (numpy/scipy restatement, complex128 like MATLAB) timed on this host."""
    import scipy.fft as sfft
    from rsp import config as C
    from oracle import chain, precompute as op
    hc = host_cpu()
    cores = hc['usable']
    pre = op.precompute(cfg, W, ang, k, C.V8_FIR)
    cube = chain.synthesize_echo(targets, cfg, pre) + chain.philox_noise(cfg, 1, 20250101)
    times = []
    with sfft.set_workers(cores):
        chain.process_cube(cube, cfg, cfar, clus, pre)   # warm-up
        t_start = time.perf_counter()
        while True:
            t0 = time.perf_counter()
            chain.process_cube(cube, cfg, cfar, clus, pre)
            times.append(time.perf_counter() - t0)
            if nframes and len(times) >= nframes:
                break
            if not nframes and (time.perf_counter() - t_start > budget_s or len(times) >= 50):
                break
    med = float(np.median(times))
    return {'value': 1.0 / med, 'unit': 'frames/s', 'cores': cores, 'kind': 'port', 'host': hc,
            'sample': '%d frames of the same %s cube, median of per-frame times (%.3f s/frame); oracle = '
                      'numpy/scipy complex128 restatement of fsf S5-S11, CFAR vectorised '
                      '(the MATLAB scalar CFAR loop fsf:192-213 would be slower)' % (len(times), name, med)}


def k3_map_bytes(P, G, B, cfar, real_bytes, rt=None):
    """Magnitude-map bytes K3 reads per frame (its stage bytes in rsp_profile_stages): with the
    reference's CFAR window (refCells 5, guardCells 10) the halo-less tiles hold only the
    P - 2 (refV + guardV) Doppler rows under test, over the tiled range columns (the first cell
    under test rounded down to 4, ceil-ish tiles of rt cells clipped to G); other windows read
    whole maps.  Restates k3_map_bytes / k3_ntiles of rsp_internal.h."""
    rt = rt if rt is not None else (64 if real_bytes == 4 else 32)
    rR, gR, rV, gV = cfar['refCells_R'], cfar['guardCells_R'], cfar['refCells_V'], cfar['guardCells_V']
    if (rR, rV, gR, gV) == (5, 5, 10, 10) and rt in (32, 64):
        rc0 = rR + gR
        ntiles = (G - rc0 - (rc0 & ~3) + rt - 1) // rt
        c0, c1 = rc0 & ~3, min(G, (rc0 & ~3) + ntiles * rt)
        return B * max(P - 2 * (rV + gV), 0) * max(c1 - c0, 0) * real_bytes
    return B * P * G * real_bytes


MFMA_F32_PEAK_TFLOPS = 157.3   # MI355X_MICROARCH.md: v_mfma_f32_16x16x4_f32 dense peak
F64_PEAK_TFLOPS = 78.6         # MI355X FP64 peak, vector and matrix alike (v_fma_f64, v_mfma_f64_16x16x4_f64)


def _music_cpu_worker(args):
    """One CPU-baseline process: synthesise its instances, wait for the others, time music_batch."""
    scene, scan, dl, N, K, M, i0, n, barrier = args
    from threadpoolctl import threadpool_limits
    from oracle import music as mu
    with threadpool_limits(1):   # one core per process: the processes are the parallelism
        Xs = np.stack([mu.synthesize(scene, N, K, dl, i, 20250101) for i in range(i0, i0 + n)])
        mu.music_batch(Xs[:2], M, scan, dl)
        barrier.wait()
        t0 = time.perf_counter()
        mu.music_batch(Xs, M, scan, dl)
        return time.perf_counter() - t0


def music_cpu_baseline(scene, scan, dl, N, K, M, per_core=48):
    """The MUSIC oracle (numpy complex128, batched eigh) on a bounded sample of instances, one
    process per usable host core (per_core instances each), all started together; rate = all
    instances / the slowest process's time."""
    import multiprocessing as mp
    hc = host_cpu()
    cores = hc['usable']
    ctx = mp.get_context('fork')
    with ctx.Manager() as mgr:
        barrier = mgr.Barrier(cores)
        with ctx.Pool(cores) as pool:
            els = pool.map(_music_cpu_worker, [(scene, scan, dl, N, K, M, c * per_core, per_core, barrier)
                                               for c in range(cores)])
    el = max(els)
    n = per_core * cores
    return {'value': n / el, 'unit': 'instances/s', 'cores': cores, 'kind': 'port', 'host': hc,
            'sample': '%d instances of the config #5 scene through oracle.music.music_batch (numpy complex128: '
                      'einsum covariance, batched LAPACK eigh, pseudo-spectrum, findpeaks), %d processes x %d '
                      'instances, one BLAS thread each, slowest %.2f s' % (n, cores, per_core, el)}


def kernel_hashes():
    """{kernel: code hash} of the built librsp.so (tools/kernel_hashes.py, written by the Makefile)."""
    p = os.path.join(PKG, 'rsp', 'kernel_hashes.json')
    if not os.path.exists(p):
        return {}
    with open(p) as f:
        return json.load(f)


def pmc_traffic(path, kernels, now=None):
    """HBM bytes per launch of the first of `kernels` a PMC traffic file (tools/pmc_traffic.py)
    holds, with its provenance.  The bytes are returned only while the file is fresh: it recorded
    the kernel's code hash when it was measured and the built kernel still has that hash;
    otherwise (kernel changed since, or a file without hashes) the traffic is None and the source
    says why.  Returns (bytes or None, file's frames per launch, source dict or None)."""
    import hashlib
    if not os.path.exists(path):
        return None, None, None
    with open(path, 'rb') as f:
        raw = f.read()
    tj = json.loads(raw)
    now = kernel_hashes() if now is None else now
    src = {'file': os.path.relpath(path, ROOT),
           'git_blob': hashlib.sha1(b'blob %d\0' % len(raw) + raw).hexdigest()}   # = git hash-object
    for k in kernels:
        if k in tj:
            measured = (tj.get('_kernel_hashes') or {}).get(k)
            src.update(kernel=k, kernel_hash_measured=measured, kernel_hash_built=now.get(k))
            src['fresh'] = measured is not None and measured == now.get(k)
            if not src['fresh']:
                src['stale_reason'] = ('the PMC file records no kernel hash' if measured is None else
                                       'the kernel changed since the PMC passes')
                return None, tj.get('_frames_per_launch'), src
            return tj[k], tj.get('_frames_per_launch'), src
    src.update(kernel=None, fresh=False, stale_reason='no entry for %s' % '/'.join(kernels))
    return None, None, src


def music_traffic(prec, n_inst, path=None, now=None):
    """k_music_cov HBM bytes of one n_inst-instance launch from the PMC passes (profiles/, made by
    tools/pmc_traffic.py over tools/music_prof.py; the file's launches held _instances_per_launch
    instances, 1024 when it does not say) and its provenance, or (None, source)."""
    tf = path or os.path.join(ROOT, 'profiles', 'pmc_traffic_music5%s.json' % ('' if prec == 'c64' else '_c128'))
    tr, _, src = pmc_traffic(tf, ['k_music_cov64', 'k_music_cov'], now=now)
    if tr is not None:
        try:
            per = json.load(open(tf)).get('_instances_per_launch', 1024)
        except (OSError, ValueError):
            per = 1024
        src['instances_per_launch_measured'] = per
        tr = tr * n_inst / float(per)
    return tr, src


def main_music(a):
    """BASELINE config #5: MUSIC_1D DOA on 64-channel x 1024-snapshot instances (MUSIC_1D.m:21-48).
    One step = one batch of --batch instances (device-resident snapshots, synthesised on the
    device) through covariance -> eig -> pseudo-spectrum -> findpeaks, peak indices to the host.
    Multi-GPU: instances sharded by rank (weak scaling), no collective."""
    rank = int(os.environ.get('RANK', 0))
    world = int(os.environ.get('WORLD_SIZE', 1))
    local = int(os.environ.get('LOCAL_RANK', 0))
    dist = None
    dev = 0 if (world == 1 or a.same_device) else local
    if world > 1:
        import torch
        import torch.distributed as dist
        if a.dist_backend == 'nccl':
            torch.cuda.set_device(dev)
            dist.init_process_group('nccl', device_id=torch.device('cuda', dev))
        else:
            dist.init_process_group('gloo')
    from rsp.music import MusicPlan, music_1d_scene
    N, K, M, I = 64, 1024, 3, a.batch
    scene, scan, dl = music_1d_scene()
    plan = MusicPlan(N, K, M, scan, dl, max_batch=I, device=dev, precision=a.precision)
    f64 = a.precision == 'c128'
    mfma_peak = F64_PEAK_TFLOPS if f64 else MFMA_F32_PEAK_TFLOPS
    valu_peak = F64_PEAK_TFLOPS if f64 else MFMA_F32_PEAK_TFLOPS
    ring = [plan.device_alloc(I) for _ in range(2)]   # 2 x 1 GiB (c128) > Infinity Cache
    for r, d in enumerate(ring):
        plan.synthesize_device(d, scene, I, inst0=(rank * 2 + r) * I)
    peaks = np.zeros((I, M), np.int32)
    npk = np.zeros(I, np.int32)
    eig = np.zeros((I, N), np.float64) if a.want_eig else None
    spec = np.zeros((I, len(scan)), np.float64) if a.want_spectrum else None

    def step(i):
        if a.want_eig:   # all N eigenvalues back with the peaks: the full eigensolver
            plan.eig_device(ring[i % 2], I, eig, peaks, npk)
        elif a.want_spectrum:   # P_dB back with the peaks
            plan.spectrum_device(ring[i % 2], I, spec, peaks, npk)
        else:
            plan.peaks_device(ring[i % 2], I, peaks, npk)

    for i in range(a.warmup):
        step(i)
    if dist is not None:
        dist.barrier()
    t0 = time.perf_counter()
    for i in range(a.steps):
        step(i)
    if dist is not None:
        dist.barrier()
    el = time.perf_counter() - t0
    if dist is not None:
        import torch
        t = torch.tensor([el], dtype=torch.float64, device='cuda' if a.dist_backend == 'nccl' else 'cpu')
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    census = rank_census(dist, dev) if dist is not None else None
    out = None
    if rank == 0:
        pr = plan.profile(ring[0], I, iters=a.profile_iters,
                          what='eigenvalues' if a.want_eig else ('spectrum' if a.want_spectrum else 'peaks'))
        n_fast = plan.fast_count()   # instances of the profiled launch on the fast path (0 with --want-eig)
        flops = 8.0 * N * (N + 1) / 2 * K * I   # Hermitian X X^H: N(N+1)/2 entries x K complex MACs
        cov_tf = flops / (pr['cov_ms'] * 1e-3) / 1e12
        bytes_ = (16.0 if f64 else 8.0) * N * K * I
        eig_flops = (16.0 / 3.0 * N ** 3 + 8.0 * M * N * N + 8.0 * len(scan) * M * N) * I
        sfx = '64' if f64 else ''
        stages = [{'stage': 'k_music_cov' + sfx, 'ms_per_launch': pr['cov_ms'], 'instances_per_launch': I,
                   'alg_flops_per_launch': flops, 'achieved_TFLOPs': cov_tf,
                   'achieved_GBps': bytes_ / (pr['cov_ms'] * 1e-3) / 1e9},
                  {'stage': 'k_music_eig' + sfx, 'ms_per_launch': pr['eig_ms'], 'instances_per_launch': I,
                   # the reference's eig(R) as a flop model -- complex Householder tridiagonalisation
                   # 16/3 N^3, back-transform of the M signal vectors 8 M N^2, pseudo-spectrum 8 n_scan
                   # M N -- not the work this kernel does: on the fast path it finds the signal
                   # subspace by block power iteration (a few A^2 X products of 64 x 64 x M)
                   'ref_eig_equiv_flops_per_launch': eig_flops,
                   'ref_eig_equiv_TFLOPs': eig_flops / (pr['eig_ms'] * 1e-3) / 1e12,
                   'fast_path_instances': n_fast,
                   'note': ('one 256-thread workgroup per instance, the matrix in registers (quad = column): '
                            'the signal subspace by block power iteration with a proven 1e-12 subspace bound '
                            '(%d of %d instances), else Householder + multisection + inverse iteration; then the '
                            'spectrum and findpeaks, all in double' % (n_fast, I) if f64 else
                            'one wave per instance, Householder + bisection + inverse iteration + spectrum in '
                            'single') + '; latency-bound (neither HBM nor MFMA), see DESIGN.md'}]
        dom = max(stages, key=lambda st: st['ms_per_launch'])
        mtraffic = music_traffic(a.precision, I)
        eig_tf = stages[1]['ref_eig_equiv_TFLOPs']
        out = {'metric': 'MUSIC_1D DOA instances/sec, 64ch x 1024 snapshots (BASELINE config #5)' +
                         (', all N eigenvalues returned (full eigensolver)' if a.want_eig else
                          (', pseudo-spectrum returned' if a.want_spectrum else '')),
               'value': I * a.steps * world / el, 'unit': 'instances/s', 'n_gpus': world, 'steps': a.steps,
               'warmup': a.warmup, 'ms_per_step': el / a.steps * 1e3, 'higher_is_better': True, 'scaling': 'weak',
               'vs_baseline': None, 'dtype': 'fp64 (complex128)' if f64 else 'fp32 (complex64)',
               'data': 'synthetic (device Philox snapshots, MUSIC_1D.m scene: -10/-30/60 deg, 10 dB measured)',
               'config': {'workload': 'BASELINE config #5: N=64 K=1024 M=3 scan=200, %d instances per step' % I +
                                      ('; eigenvalues (N per instance) and peaks returned' if a.want_eig else
                                       ('; P_dB (200 per instance) and peaks returned' if a.want_spectrum else
                                        '; peak indices returned')),
                          'parallelism': 'instance-sharded x%d' % world},
               'roofline': {'bound': 'mfma' if dom is stages[0] else 'valu', 'kernel': dom['stage'],
                            'achieved': dom['achieved_TFLOPs'] if dom is stages[0] else eig_tf,
                            'peak': mfma_peak if dom is stages[0] else valu_peak, 'unit': 'TFLOP/s',
                            'frac': (dom['achieved_TFLOPs'] if dom is stages[0] else eig_tf) /
                                    (mfma_peak if dom is stages[0] else valu_peak),
                            'traffic': mtraffic[0] if dom is stages[0] else None,
                            'traffic_source': mtraffic[1] if dom is stages[0] else None,
                            'kernel_ms': dom['ms_per_launch'],
                            'timing': 'HIP events on the plan stream, %d launches' % a.profile_iters,
                            'note': 'the dominant kernel of the step; k_music_cov%s: %.3f of the %s MFMA peak; '
                                    'k_music_eig: %.3f ms (the reference eig() model at %.3f of the vector peak)' % (
                                        '64' if f64 else '', cov_tf / mfma_peak, 'f64' if f64 else 'f32',
                                        pr['eig_ms'], eig_tf / valu_peak),
                            'stages': stages},
               'cpu_baseline': music_cpu_baseline(scene, scan, dl, N, K, M) if (world == 1 and not a.no_cpu_baseline)
               else None}
        if census is not None:
            out['distributed'] = census
    for d in ring:
        plan.device_free(d)
    plan.close()
    if dist is not None:
        dist.destroy_process_group()
    if out is not None:
        print(json.dumps(out))


def main_per_call(a):
    """Latency of the literal drop-in: `final_targets = fun_process_single_frame(targets, ...)` once
    per frame (fsf:13), as the v8 frame loop calls it and times it with tic/toc (v8:162,177,191-194).
    Each step is ONE synchronous rsp_process_targets call through the C ABI, exactly what the MEX
    gateway's rsp_mex('frame', ...) makes: on-device S4/S4.1 synthesis of the frame from the target
    list, S5-S9 on the device, S10/S11 on the host, the final targets copied out.  The targets
    evolve per frame (v8:170-173).  value = calls / s over the --steps timed calls."""
    import ctypes as ct
    from rsp import config as C, _abi
    from rsp.precompute import precompute
    from rsp.plan import Plan
    cfg, cfar, clus, W, ang, k = C.named_config(a.config)
    pre = precompute(cfg, W, ang, k, C.V8_FIR)
    plan = Plan(cfg, cfar, clus, pre, device=0, frames_per_launch=1, precision=a.precision)
    sz = plan.sizes
    targets = scene(cfg)
    cap = 4096
    tbuf = (_abi.Target * cap)()
    o = _abi.FrameOut()
    o.dets, o.dets_cap, o.targets, o.targets_cap = None, 0, ct.cast(tbuf, ct.POINTER(_abi.Target)), cap
    lib = _abi.lib()
    seqs = []
    tg = targets
    for i in range(a.warmup + a.steps):
        seqs.append(Plan._targets_in(tg))
        tg = C.evolve_targets(tg, cfg)
    ntg = len(targets)

    def call(i):
        _abi.check(lib.rsp_process_targets(plan.h, seqs[i], ntg, i + 1, 20250101, 1.0, ct.byref(o)))

    for i in range(max(a.warmup, 3)):
        call(i % len(seqs))
    times = []
    n_targets = 0
    t_all = time.perf_counter()
    for i in range(a.warmup, a.warmup + a.steps):
        t0 = time.perf_counter()
        call(i)
        times.append(time.perf_counter() - t0)
        n_targets += o.n_targets
    el = time.perf_counter() - t_all
    ms = np.array(times) * 1e3
    # the device stages of one frame in isolation (HIP events, F = 1), for the roofline object
    d_cube = plan.device_alloc(plan.cube_bytes)
    plan.synthesize_device(d_cube, targets, frame_idx=1)
    plan.sync()
    prof = plan.profile_stages([d_cube], iters=a.profile_iters)
    # the call's own S4 + S4.1 synthesis (fsf:45-88) is a device stage of the call too
    prof = [plan.profile_synthesis(d_cube, targets, iters=a.profile_iters)] + prof
    plan.device_free(d_cube)
    stages = [{'stage': pr['stage'], 'ms_per_launch': pr['ms'], 'frames_per_launch': pr['frames'],
               'alg_bytes_per_launch': pr['bytes'], 'achieved_GBps': pr['bytes'] / (pr['ms'] * 1e-3) / 1e9}
              for pr in prof]
    dom = max(stages, key=lambda s: s['ms_per_launch'])
    cells = sz.B * sz.G * sz.P
    cfg_no = {'x2': '2', 'x4': '4', 'plumbing': '1'}.get(a.config, '-')
    out = {'metric': 'per-call latency of rsp_process_targets (one synchronous fun_process_single_frame frame), '
                     '%dch×%dbeam×%dsamp×%dpulse' % (sz.C, sz.B, sz.N, sz.P),
           'value': a.steps / el, 'unit': 'frames/s', 'n_gpus': 1, 'steps': a.steps, 'warmup': a.warmup,
           'ms_per_step': el / a.steps * 1e3, 'higher_is_better': True, 'scaling': 'weak', 'vs_baseline': None,
           'dtype': 'fp64 (complex128)' if a.precision == 'c128' else 'fp32 (complex64)',
           'data': 'synthetic (device S4 synthesis + Philox noise of the v8_2 targets inside every call)',
           'per_call_ms': {'median': float(np.median(ms)), 'mean': float(ms.mean()), 'min': float(ms.min()),
                           'p10': float(np.percentile(ms, 10)), 'p90': float(np.percentile(ms, 90)),
                           'max': float(ms.max())},
           'cells_per_s': a.steps / el * cells,
           'config': {'workload': 'BASELINE config #%s: %s C=%d B=%d N=%d P=%d G=%d, synchronous calls' % (
               cfg_no, a.config, sz.C, sz.B, sz.N, sz.P, sz.G), 'frames_per_call': 1,
               'used_samples': sz.used_samples, 'targets_reported': n_targets,
               'call': 'rsp_process_targets(plan, targets, nt, frame_idx, seed, 1.0, out) -- the C call of '
                       'rsp_mex(\'frame\', ...) (matlab/rsp_mex.c)'},
           'roofline': {'bound': 'hbm', 'kernel': dom['stage'], 'achieved': dom['achieved_GBps'],
                        'peak': HBM_PEAK_GBS, 'unit': 'GB/s', 'frac': dom['achieved_GBps'] / HBM_PEAK_GBS,
                        'traffic': None, 'kernel_ms': dom['ms_per_launch'],
                        'alg_bytes_per_launch': dom['alg_bytes_per_launch'], 'frames_per_launch': 1,
                        'timing': '%d isolated one-frame launches per stage, HIP events on the kernel stream'
                                  % a.profile_iters, 'stages': stages,
                        'device_ms_per_frame': sum(s['ms_per_launch'] for s in stages)}}
    if dom['stage'] == 'k_synth':
        out['roofline']['note'] = ('k_synth is bound by its f64 VALU work (Box-Muller log/sqrt/sincos and Philox per '
                                   'sample), not by HBM: frac is its cube store rate against the HBM peak')
    if not a.no_cpu_baseline:
        out['cpu_baseline'] = cpu_baseline(cfg, cfar, clus, W, ang, k, targets, nframes=a.cpu_frames, name=a.config)
    else:
        out['cpu_baseline'] = None
    plan.close()
    print(json.dumps(out))
    return 0


def main():
    a = parse()
    bad = validate_args(a)
    if bad:
        sys.stderr.write('bench.py: %s\n' % bad)
        return 2
    env_world = int(os.environ['WORLD_SIZE']) if 'WORLD_SIZE' in os.environ else None
    visible = 0
    if env_world is None and a.gpus > 1 and not a.same_device:
        visible = visible_gpus()   # no HIP in this process: it only spawns the ranks
    mode, msg = launch_mode(a.gpus, env_world, visible, a.same_device, a.dist_backend)
    if mode == 'error':
        sys.stderr.write('bench.py: %s\n' % msg)
        return 2
    if mode == 'spawn':
        return spawn_ranks(a.gpus, sys.argv[1:])
    if a.config == 'music5':
        return main_music(a)
    if a.per_call:
        return main_per_call(a)
    rank =int(os.environ.get('RANK', 0))
    world = int(os.environ.get('WORLD_SIZE', 1))
    local = int(os.environ.get('LOCAL_RANK', 0))
    dist = None
    dev = 0 if (world == 1 or a.same_device) else local
    if world > 1:
        import torch
        import torch.distributed as dist
        if a.dist_backend == 'nccl':
            torch.cuda.set_device(dev)
            dist.init_process_group('nccl', device_id=torch.device('cuda', dev))
        else:
            dist.init_process_group('gloo')

    from rsp import config as C
    from rsp.precompute import precompute
    from rsp.plan import Plan

    cfg, cfar, clus, W, ang, k = C.named_config(a.config)
    pre = precompute(cfg, W, ang, k, C.V8_FIR)
    plan = Plan(cfg, cfar, clus, pre, device=dev, frames_per_launch=a.fpl, precision=a.precision)
    sz = plan.sizes
    targets = scene(cfg)
    cube_bytes = plan.cube_bytes
    if a.frames_total:   # config #3: every frame distinct, frame ids global across the ranks
        share = [(a.frames_total * r // world, a.frames_total * (r + 1) // world) for r in range(world)]
        f0, f1 = share[rank]
        nring = f1 - f0
    else:
        f0, nring = 1000 * rank, a.ring
    ring = [plan.device_alloc(cube_bytes) for _ in range(nring)]
    tg = targets
    for _ in range(f0 if a.frames_total else 0):   # the scene evolved to this rank's first frame
        tg = C.evolve_targets(tg, cfg)
    for i, p in enumerate(ring):
        plan.synthesize_device(p, tg, frame_idx=1 + i + f0, seed=20250101 + (0 if a.frames_total else rank))
        tg = C.evolve_targets(tg, cfg)
    plan.sync()
    hring = []
    if a.e2e:   # host copies of the ring cubes in pinned memory
        for p in ring[:4]:
            h = plan.host_alloc(cube_bytes)
            cube = plan.host_cube(h)
            cube[...] = plan.device_download(p, cube.size, plan.cdtype).reshape(cube.shape, order='F')
            hring.append(h)

    nfr = max(a.warmup, 2 * NLANES, WARM_MIN, a.steps) * a.fpl   # the queue's argument lists, built before timing
    seq_cubes = [ring[i % len(ring)] for i in range(nfr)]
    # --want-rdm: a ring of (lanes + 1) x fpl device RD maps; frame i writes map i mod len.  A map
    # comes round again only after the batch that wrote it has been harvested (rsp_enqueue_device_rdm)
    rdm_ring = [plan.device_alloc(sz.rdm_elems * sz.elem_bytes) for _ in range((NLANES + 1) * a.fpl)] \
        if a.want_rdm else []
    seq_rdms = [rdm_ring[i % len(rdm_ring)] for i in range(nfr)] if a.want_rdm else None

    def run(nbatches, base):   # nbatches full batches of fpl frames
        n = nbatches * a.fpl
        if a.e2e:
            for i in range(n):
                plan.enqueue_host(hring[i % len(hring)], base + i)
        else:
            plan.enqueue_many(seq_cubes[:n], range(base, base + n), rdms=seq_rdms[:n] if a.want_rdm else None)
        plan.drain()

    def run_all():   # config #3: each of this rank's frames once
        plan.enqueue_many(ring, range(1 + f0, 1 + f0 + len(ring)),
                          rdms=[rdm_ring[i % len(rdm_ring)] for i in range(len(ring))] if a.want_rdm else None)
        plan.drain()

    # warm-up: every lane (stream) with full batches, and >= WARM_MIN batches so that the clocks
    # and power state have settled before the timed region, whatever --warmup says
    warm_batches = max(a.warmup, 2 * NLANES, WARM_MIN)
    run(warm_batches, 0)
    plan.results_rows(clear=True)

    if dist is not None:
        dist.barrier()
    plan.sync()
    plan.set_stage_timing(a.stage_timing)   # optional live HIP events around K1/K2/K3 of every batch
    t0 = time.perf_counter()
    if a.frames_total:
        run_all()
    else:
        run(a.steps, 1)
    # every frame's final targets as packed rows (frame_idx, Range, Velocity, Angle, Power), one
    # C call; the same payload the multi-GPU gather moves
    rows = plan.results_rows(clear=True)
    if dist is not None:
        # the one collective: gather every rank's detection list (RCCL over xGMI)
        from rsp.dist import gather_rows
        counts, bufs = gather_rows(rows, rank, world, device=dev)
        n_targets_all = int(sum(np.count_nonzero(~np.isnan(b[:c, 1])) for c, b in zip(counts, bufs)))
    else:
        n_targets_all = int(np.count_nonzero(~np.isnan(rows[:, 1])))
    plan.sync()
    if dist is not None:
        dist.barrier()
    t1 = time.perf_counter()
    live = plan.stage_times()
    plan.set_stage_timing(False)
    el = t1 - t0
    if dist is not None:
        import torch
        t = torch.tensor([el], dtype=torch.float64, device='cuda' if a.dist_backend == 'nccl' else 'cpu')
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    census = rank_census(dist, dev) if dist is not None else None

    frames = a.frames_total if a.frames_total else a.steps * a.fpl * world
    fps = frames / el
    cells = sz.B * sz.G * sz.P
    out = None
    if rank == 0:
        # Roofline leg (after the timed region): each stage re-launched `profile_iters` times on
        # the same F-frame batch with HIP events on the kernel's stream, chip otherwise idle.  In the
        # timed region consecutive batches overlap on the device (lanes), so a kernel's span there
        # is shared with the neighbouring batch's kernels; --stage-timing records those spans too.
        prof = plan.profile_stages(ring, iters=a.profile_iters, d_rdms=rdm_ring[:a.fpl] if a.want_rdm else None)
        stages = []
        for lv, pr in zip(live, prof):
            st = {'stage': pr['stage'], 'ms_per_launch': pr['ms'], 'frames_per_launch': pr['frames'],
                  'alg_bytes_per_launch': pr['bytes'], 'achieved_GBps': pr['bytes'] / (pr['ms'] * 1e-3) / 1e9}
            if pr['stage'] == 'k1_dbf_mtd':   # the DBF on the matrix cores: B x C complex MACs per cell
                fl = pr['frames'] * sz.B * sz.C * sz.used_samples * sz.P * 8.0
                mpk = F64_PEAK_TFLOPS if a.precision == 'c128' else 157.3
                st['alg_mfma_flops_per_launch'] = fl
                st['achieved_mfma_TFLOPs'] = fl / (pr['ms'] * 1e-3) / 1e12
                st['mfma_frac'] = st['achieved_mfma_TFLOPs'] / mpk
                st['mfma_peak_TFLOPs'] = mpk
            if lv['launches']:
                st['live_overlapped_ms_per_launch'] = lv['ms_total'] / lv['launches']
                st['live_frames_per_launch'] = lv['frames'] / lv['launches']
            stages.append(st)
        dom = max(stages, key=lambda s: s['ms_per_launch'])
        achieved = dom['achieved_GBps']
        traffic = None
        # the PMC passes of the same workload (with the RD map written: tools/pmc_pass.sh CFG PREC rdm),
        # quoted only while the kernel's code is the one they were collected on (pmc_traffic)
        tf = os.path.join(ROOT, 'profiles', 'pmc_traffic_%s_%s%s.json' % (a.config, a.precision,
                                                                         '_rdm' if a.want_rdm else ''))
        # PMC files are keyed by kernel name: stage k1_dbf_mtd runs as k1p_dbf_mtd (persistent K1,
        # power-of-two P) or k1q_dbf_mtd (factored DFT, the reference frame's P = 332)
        tr, tf_fpl, traffic_src = pmc_traffic(tf, [dom['stage']] + (['k1p_dbf_mtd', 'k1q_dbf_mtd']
                                                                    if dom['stage'] == 'k1_dbf_mtd' else []))
        if tr is not None:   # scaled from the PMC passes' frames per launch to this run's
            traffic = tr * dom['frames_per_launch'] / float(tf_fpl or 4)
            dom['pmc_traffic_bytes'] = traffic
        esz = sz.elem_bytes
        frame_alg_bytes = sz.C * sz.N * sz.P * esz + cells * esz   # cube read + RD map write
        metric = 'frames/sec + range-Doppler cells/sec, %dch×%dbeam×%dsamp×%dpulse' % (sz.C, sz.B, sz.N, sz.P)
        cfg_no = {'x2': '2', 'x4': '4', 'plumbing': '1'}.get(a.config, '-')
        if a.frames_total:
            metric += ', batch of %d independent frames sharded over %d GPU(s)' % (a.frames_total, world)
            cfg_no = '3'
        if a.e2e:
            metric += ', end to end (host cubes in pinned memory -> H2D of the used samples -> chain)'
        if a.want_rdm:
            metric += ', complex range-Doppler map of every frame written to HBM (rsp_enqueue_device_rdm)'
        steps = (a.frames_total + a.fpl - 1) // a.fpl if a.frames_total else a.steps
        out = {
            'metric': metric,
            'value': fps, 'unit': 'frames/s', 'n_gpus': world, 'steps': steps, 'warmup': a.warmup,
            'warmup_effective': warm_batches,   # untimed batches that actually ran (>= WARM_MIN)
            'ms_per_step': el / steps * 1e3, 'higher_is_better': True,
            'scaling': 'strong' if a.frames_total else 'weak',
            'vs_baseline': None,
            'dtype': 'fp64 (complex128)' if a.precision == 'c128' else 'fp32 (complex64)',
            'data': 'synthetic (device Philox noise + v8_2 targets)',
            'cells_per_s': fps * cells,
            'achieved_GBps_frame': fps * frame_alg_bytes / 1e9,   # SURVEY 8(d) bytes: cube read + RD map write
            # the algorithmic bytes this run's kernels actually move per frame (K1 + K2 + K3 stage
            # bytes; without --want-rdm the complex RD map is not written, only |RDM|)
            'alg_bytes_moved_per_frame': sum(st['alg_bytes_per_launch'] for st in stages) / dom['frames_per_launch'],
            'rdm_written': bool(a.want_rdm),
            'config': {'workload': 'BASELINE config #%s: %s C=%d B=%d N=%d P=%d G=%d' % (
                cfg_no, a.config, sz.C, sz.B, sz.N, sz.P, sz.G), 'frames_per_launch': a.fpl, 'frames_per_step': a.fpl,
                'ring': len(hring) if a.e2e else len(ring),
                'parallelism': 'frame-sharded x%d' % world, 'used_samples': sz.used_samples,
                'targets_reported': n_targets_all},
            'roofline': {'bound': 'hbm', 'kernel': dom['stage'], 'achieved': achieved, 'peak': HBM_PEAK_GBS,
                         'unit': 'GB/s', 'frac': achieved / HBM_PEAK_GBS, 'traffic': traffic,
                         'traffic_source': traffic_src,
                         'kernel_ms': dom['ms_per_launch'], 'alg_bytes_per_launch': dom['alg_bytes_per_launch'],
                         'frames_per_launch': dom['frames_per_launch'],
                         'timing': 'roofline leg: %d isolated launches per stage, HIP events on the kernel stream '
                                   '(tools/rocprof_split.py separates them from the timed region in the rocprof '
                                   'trace)' % a.profile_iters,
                         'stages': stages},
        }
        # the box's measured stream-copy rate beside the datasheet peak
        import ctypes as ct
        from rsp import _abi
        best = 0.0
        for _ in range(3):   # the best of 3 probes of 20 copies of 1 GiB (> the 256 MiB Infinity Cache)
            gbps = ct.c_double()
            if _abi.lib().rsp_hbm_copy_probe(dev, 1 << 30, 20, ct.byref(gbps)) == 0:
                best = max(best, gbps.value)
        if best > 0:
            out['roofline']['stream_copy_GBps'] = best
            out['roofline']['frac_of_stream_copy'] = achieved / best
        if a.e2e:
            out['e2e_h2d_bytes_per_frame'] = sz.C * sz.used_samples * sz.P * esz
            out['e2e_h2d_GBps'] = fps * out['e2e_h2d_bytes_per_frame'] / 1e9
        if world == 1 and not a.no_cpu_baseline:
            out['cpu_baseline'] = cpu_baseline(cfg, cfar, clus, W, ang, k, targets, nframes=a.cpu_frames, name=a.config)
        else:
            out['cpu_baseline'] = None
        if census is not None:   # what RCCL / gloo actually joined: world size, backend, each rank's GPU
            out['distributed'] = census
    for p in ring + rdm_ring:
        plan.device_free(p)
    for h in hring:
        plan.host_free(h)
    plan.close()
    if dist is not None:
        dist.destroy_process_group()
    if out is not None:
        print(json.dumps(out))


if __name__ == '__main__':
    sys.exit(main())
