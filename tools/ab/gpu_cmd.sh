set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_music.py -x -q -m gpu --timeout 200 --timeout-method thread 2>&1 | tail -2 || exit 1
for r in 1 2; do for v in base mbase; do
  if [ $v = base ]; then lib=base; else lib=exp/ab/librsp_$v.so; fi
  echo "$r $v $(AB_LIB=$([ $v = base ] || echo $lib) timeout -k 10 200 python3 -c "
import os,sys,json,runpy,io,contextlib
sys.argv=['bench.py','--config','music5','--steps','300','--no-cpu-baseline']
if os.environ.get('AB_LIB'):
    sys.path.insert(0,'radar-signal-simulation-and-target-detection_amd'); from rsp import _abi; _abi.LIB_PATH=os.environ['AB_LIB']
buf=io.StringIO()
with contextlib.redirect_stdout(buf):
    try: runpy.run_path('bench.py', run_name='__main__')
    except SystemExit as e:
        if e.code: raise
d=json.loads(buf.getvalue().strip().splitlines()[-1]); print(round(d['value']), round(d['ms_per_step'],4))
")" || exit 1
done; done
