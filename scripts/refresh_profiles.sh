# Round-end evidence in one GPU call: PMC passes -> profiles summary (used by bench.py's
# roofline.traffic), GPU tests, bench line, rocprofv3 kernel stats.  Outputs under gpurun_out/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
bash scripts/gpu_pmc.sh || exit $?
python3 scripts/pmc_summary.py gpurun_out/pmc profiles/pmc_r02.json && cp profiles/pmc_r02.json gpurun_out/pmc_r02.json || exit $?
bash scripts/gpu_check.sh
