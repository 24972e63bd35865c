set -o pipefail
O=gpurun_out/r02zr; mkdir -p $O
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
timeout -k 10 400 rocprofv3 --kernel-trace -d /tmp/rt -o run --output-format csv -- \
    python3 $R/bench.py --envs 512 --batch-size 2048 --steps 1 --warmup 1 --no-cpu-baseline > $O/prof.log 2>&1 || exit 1
f=$(ls /tmp/rt/*kernel_trace.csv | head -1)
python3 - "$f" > $O/timeline.txt <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
# find adam kernels: minibatch boundaries
adam = [i for i, r in enumerate(rows) if "adam_kernel" in r["Kernel_Name"]]
print("kernels", len(rows), "adam", len(adam))
# take a minibatch in the middle of the last iteration
a0, a1 = adam[-20], adam[-19]
t0 = int(rows[a0]["End_Timestamp"])
busy = []
for r in rows[a0 + 1:a1 + 1]:
    s, e = int(r["Start_Timestamp"]) - t0, int(r["End_Timestamp"]) - t0
    busy.append((s, e))
    print(f"{s/1e3:8.1f} {e/1e3:8.1f} {(e-s)/1e3:7.1f} q{r.get('Queue_Id', r.get('Stream_Id','?')):>3} {r['Kernel_Name'][:80]}")
# union of busy intervals
busy.sort(); tot = 0; cur = None
for s, e in busy:
    if cur is None or s > cur[1]:
        if cur: tot += cur[1] - cur[0]
        cur = [s, e]
    else:
        cur[1] = max(cur[1], e)
tot += cur[1] - cur[0]
span = int(rows[a1]["End_Timestamp"]) - t0
print(f"span {span/1e3:.1f} us, busy {tot/1e3:.1f} us, idle {(span-tot)/1e3:.1f} us")
PY
echo done
