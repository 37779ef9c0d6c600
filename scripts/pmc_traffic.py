"""Per-launch HBM traffic of a kernel from rocprofv3 FETCH_SIZE / WRITE_SIZE passes.

usage: pmc_traffic.py <fetch_run_dir> <write_run_dir> <kernel_substring>[,<kernel_substring>...] <out.json> [steps]

With several kernels: totals over all their dispatches divided by the number of steps run.

Corrections (MI355X_MICROARCH.md, HBM section): FETCH_SIZE / WRITE_SIZE are in KiB;
on gfx950 FETCH_SIZE reports half the bytes of a wide coalesced streaming read
(TCC_EA0_RDREQ x 64 B for 128-B requests), so it is doubled; WRITE_SIZE is taken as is.
The histogram kernel's loads are 256-B wave rows (64 lanes x 4 B) issued as 128-B
requests, the case the guide calibrates.
"""
import csv
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "siril-0.9_amd", "python"))
import sg_srcid  # noqa: E402


def per_dispatch(path, kernel, counter):
    vals = []
    with open(path) as f:
        for row in csv.DictReader(f):
            if kernel in row["Kernel_Name"] and row["Counter_Name"] == counter:
                vals.append(float(row["Counter_Value"]))
    if not vals:
        raise SystemExit(f"no {counter} rows for {kernel} in {path}")
    return sum(vals) / len(vals), len(vals)


def totals(path, kernel, counter):
    """sum and dispatch count of `counter` over every dispatch whose name contains `kernel`"""
    tot, n = 0.0, 0
    with open(path) as f:
        for row in csv.DictReader(f):
            if kernel in row["Kernel_Name"] and row["Counter_Name"] == counter:
                tot += float(row["Counter_Value"])
                n += 1
    return tot, n


def main():
    fdir, wdir, kernel, out = sys.argv[1:5]
    if "," in kernel:
        # several kernels of one step (registration): totals per step over `runs` executed steps
        runs = int(sys.argv[5]) if len(sys.argv) > 5 else 1
        res = {"kernels": {}, "steps_profiled": runs,
               "correction": "FETCH_SIZE x 2 (gfx950, 128-B requests tallied at 64 B), KiB -> B; calibrated for "
                             "16-B-per-lane streaming reads only (MI355X_MICROARCH.md): the raw KiB are kept"}
        rb = wb = 0.0
        for k in kernel.split(","):
            fk, nf = totals(f"{fdir}/run_counter_collection.csv", k, "FETCH_SIZE")
            wk, nw = totals(f"{wdir}/run_counter_collection.csv", k, "WRITE_SIZE")
            res["kernels"][k] = {"fetch_size_kib_raw_per_step": fk / runs, "write_size_kib_raw_per_step": wk / runs,
                                 "dispatches": [nf, nw],
                                 "read_bytes_per_step": fk * 1024 * 2 / runs, "write_bytes_per_step": wk * 1024 / runs}
            rb += fk * 1024 * 2 / runs
            wb += wk * 1024 / runs
        res["read_bytes_per_step"], res["write_bytes_per_step"] = rb, wb
        res["traffic_bytes_per_step"] = rb + wb
    else:
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
    # the kernel sources these bytes describe (bench.py attaches them only while they match)
    res["src_files"] = sg_srcid.sources_of(kernel)
    res["src_id"] = sg_srcid.source_id(kernel)
    with open(out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
