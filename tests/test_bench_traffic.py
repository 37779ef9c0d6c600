"""bench.py attaches a PMC traffic capture (profiles/traffic_*.json, scripts/pmc_traffic.py) to
its roofline only while the capture's src_id equals the digest of the kernel sources being run
(siril-0.9_amd/python/sg_srcid.py): a kernel edited after its capture drops the field and reports
traffic_stale instead of citing bytes of another build."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "siril-0.9_amd", "python"))

import bench  # noqa: E402
import sg_srcid  # noqa: E402


def _write(d, name, src_id, nbytes=17_300_000_000):
    with open(os.path.join(d, name), "w") as f:
        json.dump({"kernel": "k_stack_hist", "traffic_bytes": float(nbytes), "src_id": src_id}, f)


def test_matching_capture_attached(tmp_path):
    _write(str(tmp_path), "traffic_sigma_512x4096x4096.json", sg_srcid.source_id("k_stack_hist"))
    r = bench.roofline(4900.0, 17_213_423_616, 512, 4096, 4096, "sigma", profiles=str(tmp_path))
    assert r["traffic"] == 17_300_000_000 and "traffic_stale" not in r
    assert r["traffic_src_id"] == sg_srcid.source_id("k_stack_hist")


def test_mismatched_capture_dropped(tmp_path):
    _write(str(tmp_path), "traffic_sigma_512x4096x4096.json", "0123456789abcdef")
    r = bench.roofline(4900.0, 17_213_423_616, 512, 4096, 4096, "sigma", profiles=str(tmp_path))
    assert r["traffic"] is None and "traffic_over_algorithmic" not in r
    assert r["traffic_stale"]["capture_src_id"] == "0123456789abcdef"


def test_capture_without_id_dropped(tmp_path):
    with open(tmp_path / "traffic_sigma_512x4096x4096.json", "w") as f:
        json.dump({"kernel": "k_stack_hist", "traffic_bytes": 1.0}, f)
    r = bench.roofline(4900.0, 17_213_423_616, 512, 4096, 4096, "sigma", profiles=str(tmp_path))
    assert r["traffic"] is None and r["traffic_stale"]["capture_src_id"] is None


def test_source_id_tracks_the_kernel_file(tmp_path):
    """the id changes with any byte of the kernel's file and equals git's blob-id recipe"""
    import shutil
    for f in sg_srcid.sources_of("k_stack_hist"):
        shutil.copy(os.path.join(sg_srcid.CSRC, f), tmp_path / f)
    a = sg_srcid.source_id("k_stack_hist", csrc=str(tmp_path))
    assert a == sg_srcid.source_id("k_stack_hist")
    with open(tmp_path / "sg_stack_hist.hip", "a") as f:
        f.write("\n")
    assert sg_srcid.source_id("k_stack_hist", csrc=str(tmp_path)) != a
    (tmp_path / "x").write_bytes(b"hello\n")
    assert sg_srcid.blob_id(str(tmp_path / "x")) == "ce013625030ba8dba906f756967f9e9ca394464a"


def test_committed_captures_carry_an_id():
    """every committed capture names the sources it was taken from (older captures without an id
    are never attached)"""
    pdir = os.path.join(ROOT, "profiles")
    for name in os.listdir(pdir):
        if name.startswith("traffic_") and name.endswith(".json"):
            with open(os.path.join(pdir, name)) as f:
                t = json.load(f)
            r = {}
            bench.load_traffic(os.path.join(pdir, name), r)
            assert ("traffic_src" in r) != ("traffic_stale" in r), (name, r)
