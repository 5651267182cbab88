"""CPU-side checks: the C-ABI library loads and exports what include/flink_window.h declares, the
ctypes structs match the header, and the host-side Java-semantics helpers agree with the pinned
known answers.  No compute call reaches the GPU here."""
import ctypes
import os
import re
import subprocess

import numpy as np
import pytest

from flink_amd import _abi, keygroups
from harness import load_golden

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "flink_window.h")


def header_functions():
    src = open(HEADER).read()
    return sorted(set(re.findall(r"\b(fw_[a-z_]+)\s*\(", src)))


def test_header_declares_the_exported_set():
    assert header_functions() == sorted(_abi.EXPORTED_SYMBOLS)


def test_library_exports_every_declared_symbol():
    lib = ctypes.CDLL(_abi.LIB_PATH)
    for name in header_functions():
        assert hasattr(lib, name), name
    out = subprocess.run(["nm", "-D", "--defined-only", _abi.LIB_PATH], capture_output=True, text=True, check=True).stdout
    exported = set(re.findall(r" T (fw_[a-z_]+)", out))
    assert set(header_functions()) <= exported


def test_library_is_gfx950_code_object():
    data = open(_abi.LIB_PATH, "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in data   # the .hip_fatbin bundle id of the device code


def test_struct_layouts_match_header():
    # offsets computed by the C compiler from the header itself
    src = r'''
#include <stddef.h>
#include <stdio.h>
#include "flink_window.h"
int main(void) {
  printf("%zu %zu %zu %zu %zu %zu\n", sizeof(fw_config), offsetof(fw_config, key_capacity),
         offsetof(fw_config, ingest_mode), sizeof(fw_out), offsetof(fw_out, n_marks), sizeof(fw_stats));
  return 0;
}
'''
    import tempfile
    with tempfile.TemporaryDirectory() as d:
        c = os.path.join(d, "t.c")
        open(c, "w").write(src)
        exe = os.path.join(d, "t")
        subprocess.run(["gcc", "-I", os.path.join(ROOT, "include"), c, "-o", exe], check=True)
        vals = list(map(int, subprocess.run([exe], capture_output=True, text=True, check=True).stdout.split()))
    assert vals == [ctypes.sizeof(_abi.FwConfig), _abi.FwConfig.key_capacity.offset, _abi.FwConfig.ingest_mode.offset,
                    ctypes.sizeof(_abi.FwOut), _abi.FwOut.n_marks.offset, ctypes.sizeof(_abi.FwStats)]


def test_host_key_group_helpers_match_known_answers():
    for key, lh, mm, kg, op in load_golden("murmur_key_groups")["cases"]:
        assert keygroups.long_hash_code(key) == lh
        assert keygroups.murmur_hash(lh) == mm
        assert keygroups.assign_to_key_group(key, 128) == kg
        assert keygroups.assign_key_to_parallel_operator(key, 128, 8) == op
    for mp, p, i, s, e in load_golden("key_group_ranges")["cases"]:
        assert keygroups.compute_key_group_range_for_operator_index(mp, p, i) == (s, e)


def test_vectorised_routing_matches_scalar():
    rng = np.random.default_rng(7)
    keys = rng.integers(-(1 << 63), (1 << 63) - 1, size=20000, dtype=np.int64)
    keys[:4] = [0, -1, -(1 << 63), (1 << 63) - 1]
    v = keygroups.operator_index_np(keys, 128, 8)
    s = np.array([keygroups.assign_key_to_parallel_operator(int(k), 128, 8) for k in keys])
    assert np.array_equal(v, s)


def test_window_assigner_factories_use_java_remainder():
    from flink_amd.windowing import SlidingEventTimeWindows, TumblingEventTimeWindows
    assert TumblingEventTimeWindows.of(1000, 2300).offset == 300
    assert TumblingEventTimeWindows.of(1000, -2300).offset == -300        # Java % keeps the sign
    assert SlidingEventTimeWindows.of(24 * 3600_000, 3600_000, -8 * 3600_000 - 5).offset == -5


def test_missing_library_fails_loudly(tmp_path):
    with pytest.raises(RuntimeError, match="not built"):
        _abi.open_library(str(tmp_path / "nope.so"))


def test_snapshot_layout_constants_match_header():
    """The key-group snapshot blob layout (fw_snapshot_kg / fw_restore_kg) seen by ctypes is the
    header's: magic, header and entry word counts."""
    src = open(HEADER).read()
    defs = dict(re.findall(r"#define (FW_SNAP_[A-Z_]+)\s+(0x[0-9a-fA-F]+|\d+)", src))
    assert int(defs["FW_SNAP_MAGIC"], 0) == _abi.FW_SNAP_MAGIC
    assert int(defs["FW_SNAP_HEADER_WORDS"]) == _abi.FW_SNAP_HEADER_WORDS
    assert int(defs["FW_SNAP_ENTRY_WORDS"]) == _abi.FW_SNAP_ENTRY_WORDS
