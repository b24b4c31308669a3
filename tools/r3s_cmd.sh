set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/r3s_pytest_gpu.txt 2>&1; rc=$?; tail -3 gpurun_out/r3s_pytest_gpu.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3s_smoke.txt 2>&1 && tail -1 gpurun_out/r3s_smoke.txt || exit 1
(SM_AB_LR=1 SM_AB_B=32 timeout -k 10 300 python tools/ab.py tools/ab/rr_old.so tools/ab/rr_new.so && SM_AB_LR=1 SM_AB_B=8 SM_AB_W=3840 SM_AB_H=2160 SM_AB_D=192 timeout -k 10 300 python tools/ab.py tools/ab/rr_old.so tools/ab/rr_new.so) > gpurun_out/r3s_rr.txt 2>&1; rc=$?; cat gpurun_out/r3s_rr.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python tools/ab_staged_kernels.py tools/ab/adv_base.so tools/ab/adv_s1r8.so tools/ab/adv_s1r4.so tools/ab/adv_s2r8.so tools/ab/adv_s4r8.so > gpurun_out/r3s_adv.txt 2>&1; rc=$?; cat gpurun_out/r3s_adv.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py > gpurun_out/r3s_bench.json 2> gpurun_out/r3s_bench.err && cut -c1-400 gpurun_out/r3s_bench.json
