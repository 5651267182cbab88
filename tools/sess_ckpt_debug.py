"""Debug aid for tests/test_session_checkpoint.py: run one case through the HIP engine and the oracle and print the
first key group whose sections differ, decoded (window-contents namespaces and entries in order, merging-window-set
entries, timers).  Usage: python tools/sess_ckpt_debug.py <case index>"""
import os
import struct
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))

import test_session_checkpoint as T  # noqa: E402


def decode_state(b, nfields):
    p = 0
    out = []

    def rd(fmt):
        nonlocal p
        v = struct.unpack_from(fmt, b, p)
        p += struct.calcsize(fmt)
        return v[0] if len(v) == 1 else v
    if not b:
        return out
    out.append(("kg", rd(">i")))
    while p < len(b):
        tid, present = rd(">h"), rd(">b")
        out.append(("table", tid, present))
        if not present:
            continue
        nns = rd(">i")
        if tid == 0:
            for _ in range(nns):
                s, e = rd(">q"), rd(">q")
                ne = rd(">i")
                ents = []
                for _ in range(ne):
                    k = rd(">q")
                    f = [rd(">q") for _ in range(nfields)]
                    ents.append((k, f[1] if nfields > 1 else None))
                out.append(("ns", s, e, ents))
        else:
            if nns:
                rd(">b")
                ne = rd(">i")
                for _ in range(ne):
                    k = rd(">q")
                    m = rd(">i")
                    out.append(("mws", k, [(rd(">q"), rd(">q"), rd(">q"), rd(">q")) for _ in range(m)]))
    return out


def decode_timers(b):
    n = struct.unpack_from(">i", b, 0)[0]
    return [struct.unpack_from(">qqqq", b, 4 + 32 * i) for i in range(n)]


def main():
    from flink_amd.windowing import WindowEngine
    from oracle.oracle import OracleEngine
    case = T.CASES[int(sys.argv[1])]
    nf = len(T._layout(case[1]))
    g, _ = T._run(WindowEngine, case)
    o, _ = T._run(OracleEngine, case)
    for i in range(len(o)):
        for kg in range(T.MP):
            for part in (0, 1):
                if g[i][kg][part] != o[i][kg][part]:
                    print(f"snapshot {i} kg {kg} {'state' if part == 0 else 'timers'} differs")
                    dec = (lambda b: decode_state(b, nf)) if part == 0 else decode_timers
                    dg, do = dec(g[i][kg][part]), dec(o[i][kg][part])
                    for j in range(max(len(dg), len(do))):
                        a = dg[j] if j < len(dg) else None
                        b = do[j] if j < len(do) else None
                        print(("   " if a == b else "!! ") + f"engine {a}\n   oracle {b}")
                    return
    print("no difference")


if __name__ == "__main__":
    main()
