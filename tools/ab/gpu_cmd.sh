set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in base wl wlbar; do
  if [ $v = base ]; then lib=""; else lib=exp/ab/librsp_$v.so; fi
  AB_LIB=$lib timeout -k 10 120 python3 tools/ab/rdm_dump.py gpurun_out/rdm_$v.npy || exit 1
done
python3 -c "
import numpy as np
b=np.load('gpurun_out/rdm_base.npy')
for v in ['wl','wlbar']:
    x=np.load('gpurun_out/rdm_%s.npy'%v); d=np.abs(x-b); print(v, 'maxdiff', d.max(), 'n bad', int((d>0).sum()), 'bad beams/doppler rows', sorted(set(np.argwhere(d>0)[:,2].tolist()))[:10], len(set(map(tuple,np.argwhere(d>0)[:,[0,2]].tolist()))))
"
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_queue_paths.py tests/test_music.py -x -q --timeout 300 --timeout-method thread -k "x2 or small or p256 or rdm or x4 or music" > gpurun_out/par.log 2>&1; rc=$?; tail -3 gpurun_out/par.log; [ $rc -eq 0 ] || exit $rc
bash tools/ab/ab.sh x2 c128 head || exit 1
mv gpurun_out/ab.log gpurun_out/ab_x2.log
bash tools/ab/ab.sh x4 c128 preunit || exit 1
mv gpurun_out/ab.log gpurun_out/ab_x4.log
bash tools/pmc_pass.sh x4 c128 || exit 1
cat gpurun_out/pmc_x4_c128/pmc_traffic_x4_c128.json
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tl_base -o run -- python3 bench.py --steps 100 --no-cpu-baseline > gpurun_out/tl_base.json 2>gpurun_out/tl_base.err || exit 1
python3 tools/timeline.py gpurun_out/tl_base
timeout -k 10 300 python3 tools/ab/cusplit.py x2 c128 | tee gpurun_out/cusplit.log
bash tools/ab/ab_bench.sh "--steps 200" split64 split96 split128 || exit 1
for v in base mmerge; do
  if [ $v = base ]; then lib=""; else lib=exp/ab/librsp_$v.so; fi
  AB_LIB=$lib timeout -k 10 120 python3 tools/ab/music_dump.py gpurun_out/music_$v.npz || exit 1
done
python3 -c "
import numpy as np
a=np.load('gpurun_out/music_base.npz'); b=np.load('gpurun_out/music_mmerge.npz')
print('music mmerge: eig maxrel', np.abs(a['eig']-b['eig']).max()/np.abs(a['eig']).max(), 'db maxdiff', np.abs(a['db']-b['db']).max(), 'peaks same', bool((a['peaks']==b['peaks']).all()))
"
for r in 1 2 3; do for v in base mmerge; do
  if [ $v = base ]; then lib=""; else lib=exp/ab/librsp_$v.so; fi
  echo "$r $v $(AB_LIB=$lib timeout -k 10 120 python3 tools/music_prof.py 1024 20 c128 | cut -c1-200)"
done; done
