# End-of-session check of the in-tree library: smoke + the GPU suite.
set -o pipefail
O=gpurun_out/r02end; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo SMOKEFAIL; tail $O/smoke.log; exit 1; }
timeout -k 10 700 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > $O/t.log 2>&1 || { echo FAIL; grep -E "^FAILED|Error" $O/t.log | head -20; tail -3 $O/t.log; exit 1; }
tail -1 $O/t.log
echo done
