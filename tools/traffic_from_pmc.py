"""Regenerate profiles/traffic.json (bench.py's roofline "traffic" per launch) from the round's
rocprofv3 --pmc summaries under profiles/: HBM bytes per launch = 2 x FETCH_SIZE + WRITE_SIZE
(KB x 1024; the x2 is MI355X_MICROARCH.md's gfx950 streaming-read correction)."""
import json
import os

P = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "profiles")


def hbm(entry):
    return (2 * entry["FETCH_SIZE"] + entry["WRITE_SIZE"]) * 1024.0


def pick(d, prefix):
    keys = [k for k in d if isinstance(d[k], dict) and prefix in k]
    assert len(keys) == 1, (prefix, keys)
    return d[keys[0]]


note = "HBM bytes per launch: 2 x FETCH_SIZE + WRITE_SIZE (KB x 1024), rocprofv3 --pmc, gfx950; source: {}"
out = {}
m6 = json.load(open(os.path.join(P, "r06", "r06_pmc_mat32_y.json")))
out["materialised_bf16_32_L4_r4_n1"] = {
    "build_hbm_bytes_per_launch": hbm(pick(m6, "k_build_bf16_2b")),
    "lookup_hbm_bytes_per_launch": hbm(pick(m6, "k_lookup_tile")),
    "note": note.format("profiles/r06/r06_pmc_mat32_y.json (round-6 last tree; DVC_BRICKED level 0)")}
mp = json.load(open(os.path.join(P, "r06", "r06_pmc_mat32_convc1.json")))
out["materialised_bf16_32_L4_r4_n1_convc1_fused"] = {
    "lookup_hbm_bytes_per_launch": hbm(pick(mp, "k_lookup_tile")),
    "note": note.format("profiles/r06/r06_pmc_mat32_convc1.json (round 6, tree 6665544; k_lookup_tile<PROJ>, "
                        "DVC_BRICKED level 0)")}
f = json.load(open(os.path.join(P, "r06", "r06_pmc_fused128_y.json")))
out["fused_bf16_128_L2_r4_n1"] = {
    "lookup_hbm_bytes_per_launch": hbm(pick(f, "k_fused_box<")),
    "note": note.format("profiles/r06/r06_pmc_fused128_y.json (round-6 last tree: 8x4x1 box group, masked window writes)")}
f32 = json.load(open(os.path.join(P, "r06", "r06_pmc_fused128_fp32_y.json")))
out["fused_fp32_128_L2_r4_n1"] = {
    "lookup_hbm_bytes_per_launch": hbm(pick(f32, "k_fused_box_f32")),
    "note": note.format("profiles/r06/r06_pmc_fused128_fp32_y.json (round-6 last tree; k_fused_box_f32)")}
fp = json.load(open(os.path.join(P, "r03", "r03_pmc_fused128_convc1.json")))
out["fused_bf16_128_L2_r4_n1_convc1_fused"] = {
    "lookup_hbm_bytes_per_launch": sum(hbm(pick(fp, k)) for k in ("k_otf_keys", "k_fused_proj", "k_rows_to_channels")),
    "note": note.format("profiles/r03/r03_pmc_fused128_convc1.json") + " (k_otf_keys + k_fused_proj + k_rows_to_channels; "
                                                                      "round 3, kernels unchanged since)"}
old = json.load(open(os.path.join(P, "traffic.json")))
for k, v in old.items():   # keep entries no round-6 pass replaced, as they were
    if k not in out:
        out[k] = v
json.dump(out, open(os.path.join(P, "traffic.json"), "w"), indent=1)
print(json.dumps(out, indent=1))
