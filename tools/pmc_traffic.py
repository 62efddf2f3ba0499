"""Per-launch HBM traffic of a kernel from rocprofv3 PMC passes (FETCH_SIZE / WRITE_SIZE, KB).

gfx950 correction (MI355X_MICROARCH.md §HBM): FETCH_SIZE reads exactly half of the bytes of
wide coalesced streaming reads, so read bytes = 2 x FETCH_SIZE x 1024; WRITE_SIZE is exact for
16-B stores.  Other access widths are uncalibrated (noted in the output).

    python tools/pmc_traffic.py <prof dir> <kernel substring> <config> <n_rows> <spp> <path> <out.json> [walk]

Pass the kernel substring `k_megakernel<false, false` to leave out bench.py's counting passes
(the STATS=true instantiation) and average only the timed launches.
"""
import csv
import glob
import json
import sys


def mean_counter(d, counter, kname):
    vals = []
    for f in glob.glob(f"{d}/*counter_collection.csv") + glob.glob(f"{d}/*/*counter_collection.csv"):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] == counter and kname in r["Kernel_Name"]:
                vals.append(float(r["Counter_Value"]))
    return sum(vals) / len(vals) if vals else None


if __name__ == "__main__":
    d, kname, config, n_rows, spp, path, out = sys.argv[1:8]
    walk = sys.argv[8] if len(sys.argv) > 8 else "ordered"
    fetch = mean_counter(d, "FETCH_SIZE", kname)
    write = mean_counter(d, "WRITE_SIZE", kname)
    rd = 2 * fetch * 1024
    wr = write * 1024
    res = {
        "config": config, "n_rows": int(n_rows), "spp": int(spp), "path": path, "kernel": kname,
        "fetch_size_kb": fetch, "write_size_kb": write,
        "hbm_read_bytes_per_launch": rd, "hbm_write_bytes_per_launch": wr,
        "hbm_bytes_per_launch": rd + wr,
        "note": "read = 2 x FETCH_SIZE (gfx950 correction for wide coalesced reads; node loads are 16-B "
                "dwordx4, rng/accum dword/dwordx4); write = WRITE_SIZE; averaged over the profiled launches",
        "source": d,
        "walk": walk,
    }
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res))
