# config #5 at 4096 instances per launch: hashed PMC traffic of that launch, then the bench line
set -o pipefail
export TMPDIR=/tmp
m=gpurun_out/pmc_music5_c128; rm -rf $m; mkdir -p $m
timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $m/fetch -o run -- python3 tools/music_prof.py 4096 5 > $m/fetch.log 2>&1 || exit $?
timeout -k 10 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $m/write -o run -- python3 tools/music_prof.py 4096 5 > $m/write.log 2>&1 || exit $?
PMC_DRIVER=tools/music_prof.py python3 tools/pmc_traffic.py $m/fetch $m/write $m/pmc_traffic_music5_c128.json 4096 5 > /dev/null || exit 1
cp $m/pmc_traffic_music5_c128.json profiles/pmc_traffic_music5_c128.json
timeout -k 10 300 python3 bench.py --config music5 > gpurun_out/r05x_bench_music5.json 2> gpurun_out/r05x_bench_music5.err || exit $?
cut -c1-400 gpurun_out/r05x_bench_music5.json
