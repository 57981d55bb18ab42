#!/bin/bash
# Full GPU suite + smoke.
set -o pipefail
O=gpurun_out/r3v
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests/ -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/t3.log 2>&1; tail -4 $O/t3.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -3 $O/smoke.log
