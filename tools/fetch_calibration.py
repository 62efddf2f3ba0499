"""Calibrate rocprofv3's FETCH_SIZE on gfx950 for the display kernel's access shapes (round-5
verdict item 6; MI355X_MICROARCH.md's x2 correction is stated for 16-B-per-lane streaming reads
only).  Two steps, both on the GPU box:

    rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/fetchcal -o fc -- \
        python3 tools/fetch_calibration.py run
    python3 tools/fetch_calibration.py report gpurun_out/fetchcal [profiles/r05/dn_rocprof] [out.json]

`run` reads 1 GiB once in each shape -- 4 B per lane (one float: the depth buffer), 12 B per lane
(three consecutive floats: the first-hit normals), 16 B per lane (one float4: the accumulator) --
through k_read_pattern<bpl> (cpt_measure_read_pattern), buffers far past the 256 MiB Infinity
Cache.  `report` divides each kernel's FETCH_SIZE x 1024 by its known bytes, then restates the
display kernel's measured read with the factor of its own access mix (k_denoise_rows reads, per
pixel, 16 B accumulator + 12 B normal + 4 B depth + 12 B mix = 44 B).
"""
import csv
import glob
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

BYTES = 1 << 30
SHAPES = (4, 12, 16)


def run():
    import torch  # noqa: F401  (one HIP runtime per process: torch's)
    from cpppathtracer_amd import Renderer
    with Renderer(0) as r:
        for bpl in SHAPES:
            gbps = r.measure_read_pattern(bpl, BYTES, 1)
            print(json.dumps({"bytes_per_lane": bpl, "bytes": BYTES, "gbps": round(gbps, 1)}), flush=True)


def fetch_by_kernel(d):
    out = {}
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for row in csv.DictReader(open(f)):
            if row["Counter_Name"] == "FETCH_SIZE":
                out.setdefault(row["Kernel_Name"], []).append(float(row["Counter_Value"]))
    return out


def report(d, dn_dir=None, out_json=None):
    fetched = fetch_by_kernel(d)
    res = {"bytes_per_kernel": BYTES, "shapes": {}}
    for bpl in SHAPES:
        k = [v for n, v in fetched.items() if f"k_read_pattern<{bpl}>" in n]
        if not k:
            raise SystemExit(f"no k_read_pattern<{bpl}> in {d}")
        fs = sum(k[0]) / len(k[0])
        res["shapes"][bpl] = {"fetch_size_kb": fs, "counted_bytes": fs * 1024, "factor": round(BYTES / (fs * 1024), 4)}
    if dn_dir:
        # the display kernel (device frame only): per pixel 16 B accumulator + 12 B normal + 4 B depth
        # + 12 B mix read; FETCH_SIZE as measured, restated with each shape's own factor
        dn = [v for n, v in fetch_by_kernel(dn_dir).items() if "k_denoise_rows<false>" in n]
        if dn:
            fs = sum(dn[0]) / len(dn[0])
            f = {b: res["shapes"][b]["factor"] for b in SHAPES}
            per_px = {16: 16, 12: 24, 4: 4}   # the accumulator; normal + mix (12 B each); depth
            mix_factor = sum(per_px[b] * f[b] for b in per_px) / sum(per_px.values())
            alg = 1920 * 1072 * 44   # 16 + 12 + 4 + 12 B read per pixel of the 1920 x 1072 launch
            res["k_denoise_rows"] = {
                "fetch_size_kb": fs,
                "read_bytes_x2_correction": fs * 1024 * 2,
                "read_bytes_calibrated": fs * 1024 * mix_factor,
                "calibrated_factor_for_its_mix": round(mix_factor, 4),
                "algorithmic_read_bytes": alg,
                "ratio_calibrated_to_algorithmic": round(fs * 1024 * mix_factor / alg, 4),
            }
    print(json.dumps(res, indent=1))
    if out_json:
        with open(out_json, "w") as fh:
            json.dump(res, fh, indent=1)


if __name__ == "__main__":
    if sys.argv[1] == "run":
        run()
    else:
        report(sys.argv[2], sys.argv[3] if len(sys.argv) > 3 else None, sys.argv[4] if len(sys.argv) > 4 else None)
