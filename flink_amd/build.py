"""In-tree build of the HIP engine (gfx950) and of the CPU parity oracle.

`build_all()` is what __graft_entry__.build() runs.  The engine is compiled with hipcc straight into
flink_amd/lib/libflink_window.so so the shared object travels with the repository snapshot.
"""
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
LIB_DIR = os.path.join(HERE, "lib")
ENGINE_SO = os.path.join(LIB_DIR, "libflink_window.so")
ORACLE_DIR = os.path.join(ROOT, "oracle")

HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = "gfx950"
ENGINE_SOURCES = ["fw_engine.hip"]
ENGINE_DEPS = ["java_semantics.h", os.path.join("..", "..", "include", "flink_window.h"), "flink_kg_format.h", "fw_decode.hip",
               "fw_session.hip", "fw_list.hip"]


def _stale(target, deps):
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def build_engine(force=False, verbose=False):
    os.makedirs(LIB_DIR, exist_ok=True)
    srcs = [os.path.join(CSRC, s) for s in ENGINE_SOURCES]
    deps = srcs + [os.path.join(CSRC, d) for d in ENGINE_DEPS]
    if not force and not _stale(ENGINE_SO, deps):
        return ENGINE_SO
    cmd = [HIPCC, f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-shared", "-munsafe-fp-atomics",
           "-Wall", "-o", ENGINE_SO] + srcs
    if verbose:
        print(" ".join(cmd))
    subprocess.run(cmd, check=True, cwd=CSRC)
    return ENGINE_SO


def build_oracle(verbose=False):
    cmd = ["make", "-C", ORACLE_DIR, "-s"]
    if verbose:
        print(" ".join(cmd))
    subprocess.run(cmd, check=True)
    return os.path.join(ORACLE_DIR, "build", "libfw_oracle.so")


def build_all(force=False, verbose=False):
    build_engine(force=force, verbose=verbose)
    build_oracle(verbose=verbose)


if __name__ == "__main__":
    build_all(force=True, verbose=True)
