"""Staged / transformed input pixels per output pixel of every K-streamed tile layer (VERDICT r5
item 2): a block stages the GroupNorm+SiLU-transformed halo of its output tile for every 32-channel
input chunk, and each of the Cout / NB channel blocks of one pixel tile stages the same halo again.

    python tools/tile_staging_ratio.py [ops.json]   # ops.json: tools/profile_ops.py --json output (adds us)

ratio = halo slots x (Cout / NB) / output pixels (min: distinct source pixels per output pixel); halo slots = (TR + 2)(TW + 2) at stride 1 (the
upsample layers stage at output resolution), (2 TR + 1)(2 TW + 1) at stride 2 (conv_tile.hip
staging geometry).
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import gen_shapes as G  # noqa: E402


def main():
    net = json.load(open(G.NETCFG))["network"]["args"]
    tabs = json.load(open(G.TUNING))["tables"]
    t = [x for x in tabs if x["num_samples"] == 16448 and x["lane_batch"] == 16][0]
    us = {}
    if len(sys.argv) > 1:
        for o in json.load(open(sys.argv[1])):
            us[o["name"].split("[")[0]] = o["avg_ms"] * 1e3
    print(f"{'layer':16s} {'cfg':>4s} {'tile':>7s} {'NB':>3s} {'Cout/NB':>7s} {'halo':>5s} {'ratio':>6s} {'min':>5s} {'us':>6s}")
    tot = 0.0
    for c in G.convs(net, t["num_samples"]):
        k = t["kernel"].get(c["name"], "")
        if not k.startswith("tile:"):
            continue
        cfg = int(k[5:])
        wpx, wco, fp, fc = G.TILE_CFGS[cfg]
        MT, NB = wpx * fp * 16, wco * fc * 16
        TW = min(c["Wo"], MT)
        TR = min(MT // TW, c["Ho"])
        halo = (2 * TR + 1) * (2 * TW + 1) if c["s2"] else (TR + 2) * (TW + 2)
        nblk = -(-c["Cout"] // NB)
        ratio = halo * nblk / (TR * TW)
        rmin = 4.0 if c["s2"] else (0.25 if c["up"] else 1.0)   # distinct source pixels per output pixel
        u = us.get(c["name"])
        tot += u or 0.0
        print(f"{c['name']:16s} {cfg:4d} {TR:3d}x{TW:<3d} {NB:3d} {nblk:7d} {halo:5d} {ratio:6.2f} {rmin:5.2f} {u if u is not None else float('nan'):6.1f}")
    if us:
        print(f"tile layers: {tot:.1f} us per step")


if __name__ == "__main__":
    main()
