cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
B="python3 bench.py --no-extra-legs --no-cpu-baseline --no-stage-timing"
for env in "GSR_VIEWS_BATCHED=0" "GSR_VIEWS_BATCHED=1" "GSR_VIEWS_FWD_GROUPS=1" "GSR_VIEWS_FWD_GROUPS=3" "GSR_VIEWS_FWD_GROUPS=2"; do
  env $env timeout -k 10 200 $B > gpurun_out/ab.json 2> gpurun_out/ab.err || { tail -3 gpurun_out/ab.err; exit 3; }
  python3 -c "import json;d=json.load(open('gpurun_out/ab.json'));print('$env', d['value'], d['ms_per_step'])"
done
rm -rf gpurun_out/trb
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/trb -o run -- python3 bench.py --no-extra-legs --no-cpu-baseline --no-stage-timing --steps 4 > gpurun_out/trb.json 2> gpurun_out/trb.err || exit 4
python3 scripts/trace_timeline.py gpurun_out/trb auto 2 > gpurun_out/timeline_bat.txt
python3 scripts/trace_overlap.py gpurun_out/trb 200 > gpurun_out/overlap_bat.txt
echo done
