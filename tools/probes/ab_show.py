"""Print an A/B directory's bench lines (dev tool): python tools/probes/ab.show.py gpurun_out/ab_TAG"""
import glob
import json
import sys

for f in sorted(glob.glob(sys.argv[1] + "/*.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    top = [(x["kernel"].split(" (")[0], x["solo_mean_us"]) for x in d.get("roofline_top", [])]
    print(f.split("/")[-1], d["value"], d["ms_per_step"], d["phases_ms_per_step"]["train"]["gpu_ms"], top)
