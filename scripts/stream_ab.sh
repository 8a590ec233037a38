set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_render.py -m gpu > gpurun_out/t_render.log 2>&1; rc=$?; tail -3 gpurun_out/t_render.log; [ $rc -le 1 ] || exit $rc
for s in 1 2 3; do timeout -k 10 300 python bench.py --streams $s --no-cpu-baseline > gpurun_out/b_s$s.json 2> gpurun_out/b_s$s.err || exit $?; python -c "import json;d=json.load(open('gpurun_out/b_s$s.json'));print($s, d['value'], d['roofline']['avg_ms'], {k:v['avg_ms'] for k,v in d['kernels'].items()})"; done
