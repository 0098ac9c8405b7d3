"""The source stamp of libglpk_mi355x.so: a hash of the HIP / C++ sources and
headers the library is built from.  build() compiles it into the library
(gk_build_stamp()), and the loader refuses a library whose stamp is not the
stamp of the sources beside it, so a stale build can never run in place of
HEAD (on the GPU box the prebuilt library travels with the tree)."""
import hashlib
import os

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
HEADER = os.path.join(os.path.dirname(HERE), "include", "glpk_mi355x.h")
SOURCES = ["gk_kernels.hip", "gk_dual.hip", "gk_reinvert.hip", "gk_primal.hip", "gk_mip.hip", "gk_scale.hip",
           "gk_advbas.hip", "gk_tabrow.hip", "gk_panel.hip", "gk_newton.hip", "gk_comm.hip", "gk_sparse.hip",
           "gk_engine.hip", "gk_npp.cc"]
HEADERS = ["gk_internal.h", "gk_device.h", "gk_hostprof.h"]
PREFIX = "GKSTAMP:"


def stamp_inputs():
    return [os.path.join(CSRC, s) for s in SOURCES + HEADERS] + [HEADER]


def source_stamp() -> str:
    """16 hex digits of sha256 over (name, content) of every input."""
    h = hashlib.sha256()
    for p in stamp_inputs():
        h.update(os.path.basename(p).encode() + b"\0")
        with open(p, "rb") as f:
            h.update(f.read())
        h.update(b"\0")
    return h.hexdigest()[:16]


def library_stamp(lib_path: str):
    """The stamp compiled into a built library (read from its bytes, nothing
    loaded), or None."""
    try:
        with open(lib_path, "rb") as f:
            data = f.read()
    except OSError:
        return None
    i = data.find(PREFIX.encode())
    if i < 0:
        return None
    return data[i + len(PREFIX):i + len(PREFIX) + 16].decode(errors="replace")
