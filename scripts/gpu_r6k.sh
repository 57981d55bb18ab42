#!/bin/bash
# Round-end check of HEAD: full GPU suite, smoke, default bench line.
set -o pipefail
O=gpurun_out/${TAG:-r6k}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/ -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cut -c1-300 $O/bench.json
python -c "import json;d=json.load(open('$O/bench.json'));print(d['roofline']['frac'], {k:(v['avg_ms'],v.get('frac')) for k,v in d['kernels'].items()})"
