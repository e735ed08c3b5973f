#!/bin/bash
# full GPU suite + smoke + bench at the current tree
set -o pipefail
O=gpurun_out/r05_full
rm -rf $O; mkdir -p $O
timeout -k 10 1500 python -u -m pytest tests -m gpu -x -v --timeout 1300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 600 python -u bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
tail -1 $O/bench.err
