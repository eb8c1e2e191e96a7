set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_fused.py tests/test_gpu_keygen.py -x -v --timeout 240 --timeout-method thread > gpurun_out/fz_tests.txt 2>&1; echo "tests rc=$?"
tail -5 gpurun_out/fz_tests.txt
timeout -k 10 200 python3 tools/ablate.py --reps 2 --fill-modes 3 --eval-modes 7 --fused-modes 27,2,0,3,10,18 > gpurun_out/fz_ablate.txt 2>&1; cat gpurun_out/fz_ablate.txt
