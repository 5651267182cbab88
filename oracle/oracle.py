"""Python handle on the CPU parity oracle (oracle/fw_oracle.cpp).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
leg, as the checker / the timed CPU column.  The product (flink_amd) never imports this module.

Parity status: pinned by the reference's own known answers transcribed under tests/golden/
(WindowOperatorTest, TimeWindowTest, EventTimeWindowCheckpointingITCase closed forms).  The
reference itself (Java, no JDK in the image) cannot be built or run here, so there is no oracle/_ref.
"""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "build", "libfw_oracle.so")

_lib = None


def load():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            subprocess.run(["make", "-C", HERE, "-s"], check=True)
        from flink_amd import _abi  # struct layouts of the public header
        lib = ctypes.CDLL(LIB)
        _abi.declare(lib, "fwo")
        lib.fwo_clear_output.argtypes = [ctypes.c_void_p]
        lib.fwo_clear_output.restype = ctypes.c_int32
        lib.fwo_murmur_hash.argtypes = [ctypes.c_int32]
        lib.fwo_murmur_hash.restype = ctypes.c_int32
        lib.fwo_long_hash_code.argtypes = [ctypes.c_int64]
        lib.fwo_long_hash_code.restype = ctypes.c_int32
        lib.fwo_key_group.argtypes = [ctypes.c_int32, ctypes.c_int32]
        lib.fwo_key_group.restype = ctypes.c_int32
        lib.fwo_operator_index.argtypes = [ctypes.c_int32] * 3
        lib.fwo_operator_index.restype = ctypes.c_int32
        lib.fwo_key_group_range.argtypes = [ctypes.c_int32] * 3 + [ctypes.POINTER(ctypes.c_int32)] * 2
        lib.fwo_key_group_range.restype = None
        lib.fwo_window_start.argtypes = [ctypes.c_int64] * 3
        lib.fwo_window_start.restype = ctypes.c_int64
        lib.fwo_run_parallel.argtypes = [ctypes.POINTER(_abi.FwConfig), ctypes.c_int32, ctypes.c_void_p, ctypes.c_void_p,
                                         ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64, ctypes.c_int64, ctypes.c_int64,
                                         ctypes.POINTER(ctypes.c_int64)]
        lib.fwo_run_parallel.restype = ctypes.c_int64
        _lib = lib
    return _lib


def OracleEngine(config):
    """Engine factory with the WindowEngine surface, backed by the oracle."""
    from flink_amd.windowing import WindowEngine
    return WindowEngine(config, lib=load(), prefix="fwo")


def key_group_range(mp, p, i):
    s, e = ctypes.c_int32(), ctypes.c_int32()
    load().fwo_key_group_range(mp, p, i, ctypes.byref(s), ctypes.byref(e))
    return s.value, e.value


def run_parallel(config, parallelism, key, ts, value, wm_every, wm_lag, final_wm):
    """Time-able CPU job: `parallelism` subtask threads behind a key-group partitioner."""
    cs = ctypes.c_int64()
    key = np.ascontiguousarray(key, dtype=np.int64)
    ts = np.ascontiguousarray(ts, dtype=np.int64)
    value = np.ascontiguousarray(value)
    n = load().fwo_run_parallel(ctypes.byref(config), parallelism, key.ctypes.data, ts.ctypes.data, value.ctypes.data,
                                len(key), wm_every, wm_lag, final_wm, ctypes.byref(cs))
    return n, cs.value
