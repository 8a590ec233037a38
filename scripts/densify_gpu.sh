# GPU check of the densification + KNN rows: parity tests, then the micro-benchmarks
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests/test_densify.py tests/test_knn.py -q -rA > gpurun_out/densify_tests.log 2>&1
rc=$?
echo "pytest rc=$rc"
if [ $rc -eq 0 ] || [ $rc -eq 1 ]; then
  timeout -k 10 300 python scripts/densify_bench.py > gpurun_out/densify_bench.json 2> gpurun_out/densify_bench.err &&
  timeout -k 10 300 python scripts/knn_bench.py > gpurun_out/knn_bench.json 2> gpurun_out/knn_bench.err
  echo "bench rc=$?"
fi
