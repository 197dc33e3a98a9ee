#!/bin/bash
# Round-4 checks of the new boundary pieces: queue RD maps, RCCL gather, mid-capacity harvest,
# reference-frame complex single; bench --gpus N launcher; --want-rdm line.
set -o pipefail
mkdir -p gpurun_out/r04a
o=gpurun_out/r04a
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_queue_paths.py tests/test_rccl_gather.py \
  "tests/test_detection_capacity.py::test_between_readback_and_device_capacity" > $o/tests.log 2>&1 || { tail -30 $o/tests.log; exit 1; }
tail -3 $o/tests.log
timeout -k 10 600 python -u -m pytest -x -v --timeout 500 --timeout-method thread tests/test_gpu_parity.py -k "reference-c64" > $o/ref_c64.log 2>&1 || { tail -30 $o/ref_c64.log; exit 1; }
tail -3 $o/ref_c64.log
timeout -k 10 300 python3 bench.py --gpus 2 --same-device --dist-backend gloo --steps 20 --warmup 5 > $o/bench_2rank.json 2> $o/bench_2rank.err || { tail -20 $o/bench_2rank.err; exit 1; }
cut -c1-200 $o/bench_2rank.json
python3 bench.py --gpus 8 > $o/bench_8.json 2> $o/bench_8.err; echo "gpus8 rc=$?"; cat $o/bench_8.err
timeout -k 10 300 python3 bench.py --want-rdm --steps 200 --no-cpu-baseline > $o/bench_rdm.json 2> $o/bench_rdm.err || { tail -20 $o/bench_rdm.err; exit 1; }
cut -c1-300 $o/bench_rdm.json
