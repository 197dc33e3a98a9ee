set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r05a; mkdir -p $o
timeout -k 10 240 python3 bench.py --steps 500 > $o/bench.json 2> $o/bench.err || exit 1
timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > $o/bench_driver.json 2> $o/bench_driver.err || exit 1
timeout -k 10 120 python3 tools/prof_stages.py x2 50 8 c128 > $o/stages.json || exit 1
timeout -k 10 300 python3 bench.py --config music5 --no-cpu-baseline > $o/music5.json 2> $o/music5.err || exit 1
timeout -k 10 120 python3 tools/music_prof.py > $o/music_prof.txt 2>&1 || exit 1
cut -c1-300 $o/*.json; cat $o/music_prof.txt | tail -20
