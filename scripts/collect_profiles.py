"""Copy the outputs of scripts/gpu_round_profiles.sh (gpurun_out/rp) into profiles/ under a round tag.

  python3 scripts/collect_profiles.py r1

Writes profiles/<tag>_bench.json, <tag>_configs.jsonl, <tag>_encode_kernel_stats.csv,
<tag>_decode_kernel_stats.csv and <tag>_pmc_traffic.json.  The traffic file holds, per kernel, the
average per-dispatch HBM bytes from the FETCH_SIZE / WRITE_SIZE passes, corrected as
MI355X_MICROARCH.md's HBM section prescribes (FETCH_SIZE is in KiB and reports half the bytes of
a wide streaming read on gfx950, so read bytes = 2 * 1024 * FETCH_SIZE; WRITE_SIZE is exact, in KiB).
bench.py reports k_emit's entry as roofline.traffic.
"""
import collections
import csv
import glob
import json
import os
import re
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
RP = os.path.join(ROOT, "gpurun_out", "rp")
PROF = os.path.join(ROOT, "profiles")


def kname(s):
    s = re.sub(r"\(.*", "", s.replace("(anonymous namespace)::", "")).replace("void ", "").replace("sdb::", "")
    return re.sub(r"<.*", "", s).strip()


def one(pattern):
    m = glob.glob(os.path.join(RP, pattern), recursive=True)
    if not m:
        raise SystemExit("missing " + pattern)
    return m[0]


def pmc(pass_name):
    """Per-kernel mean of the counter of pass rp/pmc_<pass_name> (FETCH_SIZE or WRITE_SIZE)."""
    counter = pass_name.split("_", 1)[1] if pass_name.startswith(("bloom_", "compact_", "dec_")) else pass_name
    acc = collections.defaultdict(list)
    for r in csv.DictReader(open(one("pmc_%s/**/run_counter_collection.csv" % pass_name))):
        if r["Counter_Name"] == counter:
            acc[kname(r["Kernel_Name"])].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in acc.items()}


def main():
    tag = sys.argv[1] if len(sys.argv) > 1 else "r1"
    shutil.copy(one("bench.json"), os.path.join(PROF, tag + "_bench.json"))
    shutil.copy(one("configs.jsonl"), os.path.join(PROF, tag + "_configs.jsonl"))
    for d, name in (("enc", "encode"), ("dec", "decode"), ("bloom", "bloom"), ("compact", "compact"),
                    ("codec", "codec"), ("lookup", "lookup"), ("compress", "compress"), ("single", "single_sst")):
        m = glob.glob(os.path.join(RP, d, "**", "run_kernel_stats.csv"), recursive=True)
        if m:
            shutil.copy(m[0], os.path.join(PROF, "%s_%s_kernel_stats.csv" % (tag, name)))
    for what, name in (("enc", "encode"), ("dec", "decode")):
        f = os.path.join(RP, "sq_%s_summary.txt" % what)
        if os.path.exists(f):
            shutil.copy(f, os.path.join(PROF, "%s_pmc_sq_%s.txt" % (tag, name)))
    # HBM bytes per dispatch of the bloom, compaction and decode kernels (same corrections)
    extra = {}
    for n in ("bloom", "compact", "dec"):
        fe, wr = pmc(n + "_FETCH_SIZE"), pmc(n + "_WRITE_SIZE")
        extra[n] = {k: {"read_bytes": round(2048.0 * fe.get(k, 0.0)), "write_bytes": round(1024.0 * wr.get(k, 0.0))}
                    for k in sorted(set(fe) | set(wr)) if k.startswith("k_")}
    json.dump({"correction": "read_bytes = 2 * 1024 * FETCH_SIZE; write_bytes = 1024 * WRITE_SIZE (per dispatch)",
               "commands": "rocprofv3 --kernel-trace --pmc FETCH_SIZE | WRITE_SIZE (separate passes) -- "
                           "python3 scripts/bench_configs.py --bloom | --compact | --decode --reps 3",
               "per_dispatch": extra}, open(os.path.join(PROF, tag + "_pmc_traffic_configs.json"), "w"), indent=1)
    fetch, write = pmc("FETCH_SIZE"), pmc("WRITE_SIZE")
    batch = json.load(open(one("bench.json")))["config"]["ssts_per_gpu_per_step"]
    out = {"command": "rocprofv3 --kernel-trace --pmc FETCH_SIZE | WRITE_SIZE (separate passes) -- "
                      "python3 bench.py --steps 3 --warmup 1 --no-cpu --no-verify --single-steps 0 --stage-steps 0",
           "ssts_per_dispatch": batch,
           "correction": "read_bytes = 2 * 1024 * FETCH_SIZE (gfx950 half-count of wide reads); "
                         "write_bytes = 1024 * WRITE_SIZE",
           "per_dispatch": {}}
    for k in sorted(set(fetch) | set(write)):
        # (bench.py's own copy-ceiling probes, k_diag_*, run in the same process: not the encode)
        if not k.startswith("k_") or k.startswith("k_diag"):
            continue
        rd, wr = 2048.0 * fetch.get(k, 0.0), 1024.0 * write.get(k, 0.0)
        out["per_dispatch"][k] = {"read_bytes": round(rd), "write_bytes": round(wr), "traffic_bytes": round(rd + wr)}
    # per SST: every pipeline kernel's dispatch encodes one launch set of `batch` SSTs
    out["per_kernel"] = {k: round(v["traffic_bytes"] / batch) for k, v in out["per_dispatch"].items()}
    out["per_sst_bytes"] = sum(out["per_kernel"].values())
    json.dump(out, open(os.path.join(PROF, tag + "_pmc_traffic.json"), "w"), indent=1)
    for k, v in out["per_dispatch"].items():
        print("%-22s read %8.1f MB  write %8.1f MB" % (k, v["read_bytes"] / 1e6, v["write_bytes"] / 1e6))


if __name__ == "__main__":
    main()
