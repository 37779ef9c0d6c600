"""Per-launch HBM traffic of a kernel from rocprofv3 FETCH_SIZE / WRITE_SIZE passes.

usage: pmc_traffic.py <fetch_run_dir> <write_run_dir> <kernel_substring> <out.json>

Corrections (MI355X_MICROARCH.md, HBM section): FETCH_SIZE / WRITE_SIZE are in KiB;
on gfx950 FETCH_SIZE reports half the bytes of a wide coalesced streaming read
(TCC_EA0_RDREQ x 64 B for 128-B requests), so it is doubled; WRITE_SIZE is taken as is.
The histogram kernel's loads are 256-B wave rows (64 lanes x 4 B) issued as 128-B
requests, the case the guide calibrates.
"""
import csv
import json
import sys


def per_dispatch(path, kernel, counter):
    vals = []
    with open(path) as f:
        for row in csv.DictReader(f):
            if kernel in row["Kernel_Name"] and row["Counter_Name"] == counter:
                vals.append(float(row["Counter_Value"]))
    if not vals:
        raise SystemExit(f"no {counter} rows for {kernel} in {path}")
    return sum(vals) / len(vals), len(vals)


def main():
    fdir, wdir, kernel, out = sys.argv[1:5]
    fetch_kib, nf = per_dispatch(f"{fdir}/run_counter_collection.csv", kernel, "FETCH_SIZE")
    write_kib, nw = per_dispatch(f"{wdir}/run_counter_collection.csv", kernel, "WRITE_SIZE")
    res = {
        "kernel": kernel,
        "fetch_size_kib_raw": fetch_kib,
        "write_size_kib_raw": write_kib,
        "dispatches": [nf, nw],
        "read_bytes": fetch_kib * 1024 * 2,
        "write_bytes": write_kib * 1024,
        "correction": "FETCH_SIZE x 2 (gfx950, 128-B requests tallied at 64 B), KiB -> B",
    }
    res["traffic_bytes"] = res["read_bytes"] + res["write_bytes"]
    with open(out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
