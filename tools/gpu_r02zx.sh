# Re-entry check of HEAD: full GPU suite, smoke, default bench line.
set -o pipefail
O=gpurun_out/r02zx; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > $O/t.log 2>&1 || { echo FAIL; grep -E "^FAILED|Error" $O/t.log | head -20; tail -3 $O/t.log; exit 1; }
tail -2 $O/t.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo SMOKEFAIL; tail $O/smoke.log; exit 1; }
timeout -k 10 500 python bench.py > $O/bench.json 2>$O/bench.err || exit 1
cut -c1-400 $O/bench.json
echo done
