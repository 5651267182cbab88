"""Generates tests/golden/wire_stream.json: byte streams in Flink's network wire format with their decoded
contents, written from the format's definition (independently of the oracle and of the engine).

Per element (the sending side, paths relative to the reference root):
  SpanningRecordSerializer.addRecord   int32 big-endian length, then the serialized element
      (flink-runtime/src/main/java/org/apache/flink/runtime/io/network/api/serialization/
       SpanningRecordSerializer.java:69-92)
  StreamElementSerializer.serialize    tag 0 + int64 timestamp + value | tag 1 + value | tag 2 + int64
      watermark | tag 3 + int64 markedTime + int32 vertexId + int32 subtaskIndex
      (flink-streaming-java/src/main/java/org/apache/flink/streaming/runtime/streamrecord/
       StreamElementSerializer.java:155-178)
  TupleSerializer.serialize            the fields in order, LongSerializer (8 B) / DoubleSerializer (8 B,
      doubleToLongBits) / IntSerializer (4 B), all big-endian
      (flink-core/src/main/java/org/apache/flink/api/java/typeutils/runtime/TupleSerializer.java:120-129)

Run from the repo root:  python tests/golden/make_wire_fixture.py
"""
import json
import math
import os
import random
import struct

OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "wire_stream.json")
FMT = {"long": ">q", "double": ">d", "int": ">i"}


def element_bytes(kind, payload, fields):
    if kind == "record":
        ts, values = payload
        body = (struct.pack(">bq", 0, ts) if ts is not None else struct.pack(">b", 1))
        for f, v in zip(fields, values):
            if f == "double" and math.isnan(v):
                body += struct.pack(">Q", 0x7FF8000000000000)   # doubleToLongBits
            else:
                body += struct.pack(FMT[f], v)
    elif kind == "watermark":
        body = struct.pack(">bq", 2, payload)
    else:
        t, vertex, subtask = payload
        body = struct.pack(">bqii", 3, t, vertex, subtask)
    return struct.pack(">i", len(body)) + body


def make(name, fields, key, value, f1, n, seed):
    rng = random.Random(seed)
    stream, records, wms, lms = b"", [], [], []
    ts = 1_700_000_000_000
    for i in range(n):
        r = rng.random()
        if r < 0.03:
            wm = ts - rng.randrange(500)
            stream += element_bytes("watermark", wm, fields)
            wms.append([wm, len(records)])
        elif r < 0.04:
            lm = [ts + rng.randrange(100), rng.randrange(1 << 20), rng.randrange(64)]
            stream += element_bytes("latency", lm, fields)
            lms.append([lm[0], (lm[1] << 32) | lm[2], len(records)])
        else:
            ts += rng.randrange(3)
            has_ts = rng.random() > 0.02
            vals = []
            for j, f in enumerate(fields):
                if f == "int":
                    vals.append(rng.randrange(-(1 << 31), 1 << 31) if rng.random() < 0.3 else rng.randrange(-40, 40))
                elif f == "long":
                    # small values: their low 4 bytes look like element lengths (9, 17, 33, ...) to a scan that
                    # starts inside a record
                    vals.append(rng.choice([9, 17, 33, 25, 0, 1, -1]) if rng.random() < 0.3 else
                                rng.randrange(-(1 << 63), 1 << 63))
                else:
                    vals.append(rng.choice([0.0, -0.0, 1.5, float("inf"), float("nan"), -2.25e300]))
            rts = ts - rng.randrange(200) if has_ts else None
            stream += element_bytes("record", (rts, vals), fields)
            dec = []
            for f, v in zip(fields, vals):
                if f == "double":
                    bits = 0x7FF8000000000000 if math.isnan(v) else struct.unpack(">q", struct.pack(">d", v))[0]
                    dec.append(bits - (1 << 64) if bits >= 1 << 63 else bits)
                else:
                    dec.append(v)
            rec_ts = rts if has_ts else -(1 << 63)   # StreamRecord without timestamp: Long.MIN_VALUE
            records.append([dec[key], dec[f1] if f1 is not None else rec_ts, rec_ts, dec[value]])
    return dict(name=name, fields=fields, key=key, value=value, f1=f1, stream=stream.hex(),
                records=records, watermarks=wms, latency_markers=lms)


def main():
    sc = [make("tuple3_long", ["long", "long", "long"], 0, 2, 1, 2500, 21),
          make("tuple4_int_key_double", ["int", "long", "double", "long"], 0, 2, None, 1800, 22)]
    with open(OUT, "w") as f:
        json.dump({"generator": "tests/golden/make_wire_fixture.py", "scenarios": sc}, f, separators=(",", ":"))
    print("wrote", OUT, [len(s["stream"]) // 2 for s in sc])


if __name__ == "__main__":
    main()
