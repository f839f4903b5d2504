"""Summarise a tools/profile_ops.py --json file: total launch time and the deep-level share."""
import json
import sys

DEEP = {"downs.7", "downs.8", "downs.9", "downs.10", "mid.0", "ups.0", "ups.1", "ups.2", "ups.3", "ups.4", "ups.5", "ups.6"}
d = json.load(open(sys.argv[1]))
tot = sum(o["avg_ms"] for o in d) * 1000
deep = sum(o["avg_ms"] for o in d if ".".join(o["name"].split("[")[0].split(".")[:2]) in DEEP) * 1000
print(f"total {tot:.1f} us over {len(d)} ops, deep levels (32x16 and below) {deep:.1f} us")
