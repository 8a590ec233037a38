# rocprofv3 kernel stats of the adjacent rows' micro-benchmarks (densification, KNN, losses)
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 600 python -m pytest tests/test_losses.py -q > gpurun_out/loss_tests.log 2>&1; echo "loss tests rc=$?"
for b in densify knn loss; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$b -o run -- python3 scripts/${b}_bench.py > gpurun_out/${b}_bench_prof.json 2> gpurun_out/${b}_prof.err
  rc=$?; echo "$b prof rc=$rc"
  if [ $rc -ne 0 ]; then exit $rc; fi
done
