"""CPU: the compile-time layer-shape tables (conv_tile_cfg.h kTileShapes, conv_deep.hip kDeepShapes,
conv_strip_impl.h kStripShapes; DESIGN.md §3 "Compile-time layer shapes") agree with the measured
per-layer kernel tables (configs/conv_tuning.json) and cover every conv of the headline and config #5 plans.  A
row that drifts from the table is never wrong (the launch falls back to the generic kernel when a
field differs) but silently loses the specialisation, so the drift is caught here."""
import json
import os
import re

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(REPO, "speech-denoising-diffusion-model-2_amd", "csrc")
TUNING = os.path.join(REPO, "speech-denoising-diffusion-model-2_amd", "configs", "conv_tuning.json")
FIELDS = ("cfg", "s2", "TR", "TW", "Ho", "Wo", "CA", "CB", "Cout", "RCA", "RCB", "res", "gn", "up", "nw", "nb",
          "f16only")


def _rows(path, table):
    src = open(os.path.join(CSRC, path)).read()
    body = src[src.index(f"static constexpr ConvShape {table}[] = {{"):]
    body = body[:body.index("\n};")]
    rows = []
    for m in re.finditer(r"\{([-\d,\s]+)\},\s*//\s*(\S+)", body):
        vals = [int(v) for v in m.group(1).split(",")]
        row = dict(zip(FIELDS, vals + [0] * (len(FIELDS) - len(vals))))
        rows.append((m.group(2), row))
    return rows


def _tables():
    return {"tile": _rows("conv_tile_cfg.h", "kTileShapes"), "deep": _rows("conv_deep.hip", "kDeepShapes"),
            "strip": _rows("conv_strip_impl.h", "kStripShapes")}


def test_generic_entry_first():
    for kind, rows in _tables().items():
        assert rows[0][0] == "generic" and rows[0][1]["cfg"] == -1, kind


# row name prefix -> (num_samples, lane_batch) of the measured table the rows encode
GEOMETRIES = {"": (16448, 16), "c5:": (32832, 64)}


def _table(prefix):
    """The measured table of one geometry (the file holds one table or {"tables": [...]})."""
    tuning = json.load(open(TUNING))
    tabs = tuning["tables"] if "tables" in tuning else [tuning]
    n, lb = GEOMETRIES[prefix]
    hits = [t for t in tabs if t["num_samples"] == n and t["lane_batch"] == lb]
    assert len(hits) == 1
    return hits[0]


def _headline_table():
    return _table("")


def _split(name):
    """(geometry prefix, layer name) of a shape row's name."""
    return ("c5:", name[3:]) if name.startswith("c5:") else ("", name)


def test_rows_match_the_measured_kernel_table():
    for kind, rows in _tables().items():
        for full, r in rows[1:]:
            prefix, name = _split(full)
            kern = _table(prefix)["kernel"]
            assert name in kern, f"{kind} shape row {full} names no layer of the tuning table"
            # the config #5 rows are instantiated for fp16 only (its configured dtype)
            assert r["f16only"] == (1 if prefix else 0), full
            if kind == "tile":
                want = f"tile:{r['cfg']}"
            elif kind == "deep":
                want = f"deep:{r['cfg']}:{r['nw']}:{r['nb']}"
            else:
                want = "strip"
            assert kern[name] == want, f"{name}: shape row is {want}, tuning table says {kern[name]}"


def test_every_tuned_layer_has_exactly_one_shape():
    for prefix in GEOMETRIES:
        kern = _table(prefix)["kernel"]
        names = [_split(n)[1] for rows in _tables().values() for n, _ in rows[1:] if _split(n)[0] == prefix]
        assert sorted(names) == sorted(kern), (prefix, set(names) ^ set(kern))


def test_row_invariants():
    for kind, rows in _tables().items():
        for name, r in rows[1:]:
            assert r["Ho"] % r["TR"] == 0 and r["Wo"] % r["TW"] == 0, name
            assert (r["CA"] + r["CB"]) % 32 == 0 and r["Cout"] % 32 == 0, name
            assert r["res"] in (0, 1, 2) and (r["res"] == 2) == (r["RCA"] + r["RCB"] > 0), name
            assert not (r["s2"] and r["up"]), name
            if r["res"]:
                assert r["gn"] == 1, f"{name}: residual modes are ResnetBlock block2 convs (GroupNorm input)"
            if kind == "strip":
                assert r["TR"] == r["nb"] and r["TW"] == r["Wo"], f"{name}: strip rows encode TR = strip rows, TW = W"
            if kind == "deep":
                assert r["TR"] * r["TW"] <= r["cfg"] and r["nw"] in (4, 8) and r["nb"] in (16, 32, 64), name


def test_rows_are_the_generators_output():
    """The three tables are generated from configs/conv_tuning.json by tools/gen_shapes.py (the
    runtime's layer walk and tile rules for the kernel each measured table names): the committed
    rows are exactly its output, every field, so a re-measured table is applied by re-running it."""
    import sys
    sys.path.insert(0, os.path.join(REPO, "tools"))
    import gen_shapes
    gen = gen_shapes.generate()
    for kind, rows in _tables().items():
        assert [(n, r) for n, r in rows[1:]] == [(n, dict(r)) for n, r in gen[kind]], kind
    for kind, (path, table) in gen_shapes.TABLES.items():
        text = open(os.path.join(CSRC, path)).read()
        assert gen_shapes.splice(text, table, gen_shapes.render(gen[kind])) == text, path
