set -u
mkdir -p gpurun_out/final
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/final/tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/final/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/final/smoke.log 2>&1; rc=$?; echo "smoke rc=$rc"; tail -2 gpurun_out/final/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py > gpurun_out/final/bench.log 2>&1; rc=$?; echo "bench rc=$rc"; grep "^{" gpurun_out/final/bench.log | cut -c1-300
