# round-5 evidence pass: MUSIC PMC traffic (hashed), x2 PMC traffic, the profile round of the
# 500-step bench, the driver-command bench and the steps sweep
set -o pipefail
o=gpurun_out/r05l; mkdir -p $o
export TMPDIR=/tmp
m=gpurun_out/pmc_music5_c128; mkdir -p $m
timeout -k 10 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $m/fetch -o run -- python3 tools/music_prof.py 1024 > $m/fetch.log 2>&1 || exit $?
timeout -k 10 90 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $m/write -o run -- python3 tools/music_prof.py 1024 > $m/write.log 2>&1 || exit $?
PMC_DRIVER=tools/music_prof.py python3 tools/pmc_traffic.py $m/fetch $m/write $m/pmc_traffic_music5_c128.json 1024 > /dev/null || exit 1
bash tools/pmc_pass.sh x2 c128 || exit $?
bash tools/profile_round.sh r05 x2 c128 --steps 500 || exit $?
for k in 20 100 500; do
  timeout -k 10 240 python3 bench.py --steps $k --warmup 5 > $o/bench_steps$k.json 2> $o/bench_steps$k.err || exit $?
  cut -c1-200 $o/bench_steps$k.json
done
timeout -k 10 240 python3 bench.py --steps 20 --warmup 5 > $o/bench_steps20_b.json 2>> $o/bench_steps20.err || exit $?
timeout -k 10 240 python3 bench.py --steps 100 --warmup 5 > $o/bench_steps100_b.json 2>> $o/bench_steps100.err || exit $?
timeout -k 10 240 python3 tools/ab/steps_sweep.py x2 c128 8 > $o/steps_sweep.txt 2>&1 || exit $?
tail -20 $o/steps_sweep.txt
