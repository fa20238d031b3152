"""Shared by tests/pmc_summary.py (which records it) and bench.py (which checks it): a digest of
the product sources, so that a committed counter summary is used only for the tree it was
profiled on.  The GPU box gets a snapshot without .git, so the digest is computed from the files
themselves: the HIP kernels, the C ABI / C++ API sources, the public headers and the Makefile."""
import glob
import hashlib
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "modify-sift-gpu_amd")


def source_files():
    files = sorted(glob.glob(os.path.join(PKG, "csrc", "*")))
    files += sorted(glob.glob(os.path.join(ROOT, "include", "*.h")))
    files.append(os.path.join(PKG, "Makefile"))
    return [f for f in files if os.path.isfile(f)]


def source_digest():
    h = hashlib.sha256()
    for f in source_files():
        h.update(os.path.relpath(f, ROOT).encode())
        with open(f, "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]


def box_name():
    """The machine a profile ran on (hostname; the GPU box is a fresh pod each call)."""
    import socket
    return socket.gethostname()
