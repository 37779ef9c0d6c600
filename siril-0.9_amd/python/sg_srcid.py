"""Source identity of the kernels a PMC traffic capture describes.

profiles/traffic_*.json record the HBM bytes of a kernel as it was built when the counters were
collected (scripts/pmc_traffic.py).  Each file carries `src_id`, a digest of the kernel's source
files (their git blob ids, so `git hash-object` reproduces each part), and bench.py attaches the
traffic to its roofline only while the built sources still have that id: a kernel edited since the
capture drops the field instead of citing stale bytes.
"""
import hashlib
import os

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
CSRC = os.path.join(ROOT, "siril-0.9_amd", "csrc")

# kernel name prefix -> the source files that define it (the kernel body and the headers its
# inner loops are written in)
KERNEL_SOURCES = {
    "k_stack_hist": ["sg_stack_hist.hip", "sg_common.hpp"],
    "k_stack_reduce3": ["sg_stack.hip", "sg_common.hpp"],
    "k_stack_linfit": ["sg_stack.hip", "sg_common.hpp"],
    "k_reg_": ["sg_register.hip", "sg_fft.hpp"],
    "k_quality": ["sg_register.hip"],
}


def blob_id(path):
    """git's blob id of a file (sha1 of 'blob <size>\\0' + content)"""
    with open(path, "rb") as f:
        data = f.read()
    return hashlib.sha1(b"blob %d\0" % len(data) + data).hexdigest()


def sources_of(kernels):
    """the source files of one kernel name or a comma-separated list of them"""
    files = []
    for k in kernels.split(","):
        for prefix, fs in KERNEL_SOURCES.items():
            if k.startswith(prefix) or prefix.startswith(k):
                files += [f for f in fs if f not in files]
    if not files:
        raise KeyError(f"no source files known for kernel {kernels!r}")
    return sorted(files)


def source_id(kernels, csrc=CSRC):
    """digest over the blob ids of the kernel's source files, with the file names"""
    h = hashlib.sha1()
    for f in sources_of(kernels):
        h.update(f"{f} {blob_id(os.path.join(csrc, f))}\n".encode())
    return h.hexdigest()[:16]
