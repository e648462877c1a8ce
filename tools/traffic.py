"""Average per-dispatch HBM bytes per kernel from rocprofv3 PMC passes (tools/pmc.sh).

FETCH_SIZE is doubled: on gfx950 it reports exactly half the bytes of wide coalesced streaming reads
(MI355X_MICROARCH.md, HBM section); WRITE_SIZE is exact for 16-B-per-lane streaming stores.  Both
counters are in KB (rocprofv3 derived counters) and converted to bytes here.
Output: JSON {short_kernel_name: {"read": B, "write": B, "bytes": B, "dispatches": n}} on stdout.
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

SHORT = {
    "topk_filter_kernel": "topk_filter",
    "sparse_decode_kernel<1": "stacked_decode",
    "sparse_decode_wave2_kernel<1": "stacked_decode",
    "sparse_decode_wave_kernel<1": "stacked_decode",
    "sparse_decode_wave2_kernel<0": "sparse_decode",
    "sparse_decode_wave_kernel<0": "sparse_decode",
    "topk_sample_kernel": "topk_sample",
    "sparse_decode_kernel<0": "sparse_decode",
    "topk_select_kernel<true, true, flc::(anonymous namespace)::FlatSrc, true>": "stacked_encode_batch",
    "topk_select_kernel<true, true, flc::(anonymous namespace)::DeltaSrc, false>": "stacked_encode_delta",
    "topk_select_kernel<true, true, flc::(anonymous namespace)::FlatSrc, false>": "stacked_encode",
    "topk_select_kernel<false, true, flc::(anonymous namespace)::FlatSrc, false>": "topk_encode",
    "topk_select_kernel<true, true, flc::(anonymous namespace)::DeltaSrc>": "stacked_encode_delta",
    "topk_select_kernel<true, true, flc::(anonymous namespace)::FlatSrc>": "stacked_encode",
    "topk_select_kernel<false, true, flc::(anonymous namespace)::FlatSrc>": "topk_encode",
    "topk_select_kernel<true>": "stacked_select",
    "topk_select_kernel<false>": "topk_select",
    "topk_select_kernel<true, true>": "stacked_encode",
    "topk_select_kernel<false, true>": "topk_encode",
    "topk_select_kernel<true, false": "stacked_select",
    "topk_select_kernel<false, false": "topk_select",
    "topk_sample_select_kernel": "topk_sample_select",
    "topk_sample_gather_kernel": "topk_sample_gather",
    "tile_index_kernel": "tile_index",
    "quant_encode_kernel": "quant_encode",
    "quant_decode_kernel": "quant_decode",
    "weighted_sum_kernel": "weighted_sum",
    "sel64_select_kernel": "sel64_select",
    "sel64_emit_kernel": "sel64_emit",
    "sel64_prep_kernel": "sel64_prep",
}


def short(name):
    for k, v in SHORT.items():
        if k in name:
            return v
    return None


def collect(root, tag, counter):
    vals = defaultdict(list)
    for path in glob.glob(os.path.join(root, f"{tag}_{counter}", "**", "*counter_collection.csv"), recursive=True):
        with open(path) as f:
            for row in csv.DictReader(f):
                if row.get("Counter_Name") != counter:
                    continue
                s = short(row.get("Kernel_Name", ""))
                if s:
                    vals[s].append(float(row["Counter_Value"]))
    return vals


def main():
    root, tag = sys.argv[1], sys.argv[2]
    fetch, write = collect(root, tag, "FETCH_SIZE"), collect(root, tag, "WRITE_SIZE")
    out = {}
    for k in sorted(set(fetch) | set(write)):
        f = fetch.get(k, [])
        w = write.get(k, [])
        rd = 2.0 * 1024.0 * sum(f) / len(f) if f else None  # KB -> B, gfx950 x2 correction
        wr = 1024.0 * sum(w) / len(w) if w else None
        out[k] = {"read": rd, "write": wr, "bytes": (rd or 0.0) + (wr or 0.0), "dispatches": max(len(f), len(w)),
                  "note": "FETCH_SIZE x2 (gfx950 half-count), WRITE_SIZE as reported; KB->B"}
    json.dump(out, sys.stdout, indent=1)


if __name__ == "__main__":
    main()
