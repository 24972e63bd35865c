"""One minibatch's kernel timeline from a rocprofv3 --kernel-trace csv (dev tool): every launch
between two Adam steps of the last iteration, start / end (us from the previous Adam's end), duration,
queue, and the busy / idle time of the union.  Usage: python tools/timeline.py kernel_trace.csv [k-th from end;
-k: the k-th from the start]"""
import csv
import sys


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    back = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    adam = [i for i, r in enumerate(rows) if "adam_kernel" in r["Kernel_Name"]]
    print("kernels", len(rows), "adam", len(adam))
    a0, a1 = adam[-back], adam[-back + 1]
    t0 = int(rows[a0]["End_Timestamp"])
    busy = []
    for r in rows[a0 + 1:a1 + 1]:
        s, e = int(r["Start_Timestamp"]) - t0, int(r["End_Timestamp"]) - t0
        busy.append((s, e))
        name = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "")
        print(f"{s/1e3:8.1f} {e/1e3:8.1f} {(e-s)/1e3:7.1f} q{r.get('Queue_Id', r.get('Stream_Id', '?')):>3} {name[:90]}")
    busy.sort()
    tot, cur = 0, None
    for s, e in busy:
        if cur is None or s > cur[1]:
            if cur:
                tot += cur[1] - cur[0]
            cur = [s, e]
        else:
            cur[1] = max(cur[1], e)
    tot += cur[1] - cur[0]
    span = int(rows[a1]["End_Timestamp"]) - t0
    print(f"span {span/1e3:.1f} us, busy {tot/1e3:.1f} us, idle {(span-tot)/1e3:.1f} us")


if __name__ == "__main__":
    main()
