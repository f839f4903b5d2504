"""Compare per-layer launch times of profile_ops.py JSON dumps (family sums and per-op deltas).

    python tools/ops_cmp.py base.json new.json [--ops]
"""
import json
import sys


def fam(n):
    for k in ("deep", "tile", "strip"):
        if "[" + k in n:
            return k
    return n


def main():
    files = [a for a in sys.argv[1:] if not a.startswith("--")]
    runs = [{o["name"]: o["avg_ms"] * 1e3 for o in json.load(open(f))} for f in files]
    for f, r in zip(files, runs):
        s = {}
        for n, t in r.items():
            s[fam(n)] = s.get(fam(n), 0.0) + t
        print(f"{f}: total {sum(r.values()):.1f} us  " + "  ".join(f"{k} {v:.1f}" for k, v in sorted(s.items())))
    if "--ops" in sys.argv and len(runs) >= 2:
        base = {n.split("[")[0]: t for n, t in runs[0].items()}
        for n, t in sorted(runs[-1].items(), key=lambda kv: -kv[1]):
            b = base.get(n.split("[")[0])
            print(f"{t:8.2f} us  {'' if b is None else f'{t - b:+7.2f}'}  {n}")


if __name__ == "__main__":
    main()
