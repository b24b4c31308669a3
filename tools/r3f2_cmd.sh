set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/r3f2_pytest_gpu.txt 2>&1; rc=$?; tail -3 gpurun_out/r3f2_pytest_gpu.txt; [ $rc -eq 0 ] || { grep -E "FAILED|Error" gpurun_out/r3f2_pytest_gpu.txt | head; exit $rc; }
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3f2_smoke.txt 2>&1 && tail -1 gpurun_out/r3f2_smoke.txt || exit 1
timeout -k 10 300 python bench.py > gpurun_out/r3f2_bench.json 2> gpurun_out/r3f2_bench.err && cut -c1-200 gpurun_out/r3f2_bench.json
