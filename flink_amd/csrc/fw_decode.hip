// fw_decode.hip — GPU decode of Flink's network wire format into record columns.
// Included at the end of fw_engine.hip (uses the engine's stream, allocator and error reporting).
//
// The stream: elements back to back, each an int32 BE length then that many bytes
// (SpanningRecordSerializer.addRecord, flink-runtime/.../io/network/api/serialization/
// SpanningRecordSerializer.java:69-92); an element is StreamElementSerializer.serialize's output
// (SJ/runtime/streamrecord/StreamElementSerializer.java:155-178): tag 0 | int64 ts | tuple, tag 1 | tuple,
// tag 2 | int64 watermark, tag 3 | int64 markedTime | int32 vertexId | int32 subtaskIndex; the tuple is
// TupleSerializer.serialize's fields in order (flink-core/.../typeutils/runtime/TupleSerializer.java:120-129).
//
// Finding element boundaries is the sequential part of the receiver (one length after another,
// SpillingAdaptiveSpanningRecordDeserializer).  Here the bytes are cut into 4 KiB chunks; every chunk
// follows the length chain from each offset an element could start at (elements are shorter than
// DEC_MAXE bytes), validating every step against the lengths and tags the schema allows.  Chains from
// different offsets merge within a few elements and the ones off the boundaries die at a bad length or
// tag, so the surviving chains of a chunk nearly always leave it at one offset: the next chunk's entry,
// known without the chunks before.  The rare chunks whose survivors disagree are linked one after
// another.  A second pass walks each chunk's true chain once and decodes its elements in parallel.
#pragma once

namespace fw {

constexpr int DEC_CHUNK = 4096;    // bytes per chunk
constexpr int DEC_THREADS = 128;   // >= DEC_MAXE: one lane per candidate entry offset
constexpr int DEC_MAXE = 4 + 1 + 8 + 8 * FW_DECODE_MAX_FIELDS;   // longest element with its length prefix
constexpr int DEC_MAXEL = DEC_CHUNK / 13 + 2;   // element starts per chunk (the shortest element: 4 + 9 bytes)

struct DecSpec {
  const uint8_t* bytes;
  int64_t nbytes;
  int64_t nchunks;
  int32_t rec_ts_len, rec_len;   // element lengths (after the prefix) of records with / without timestamp
  int32_t key_off, key_int, f1_off, f1_int, val_off;   // byte offsets of fields in the tuple; int fields
  int32_t maxe;                  // candidate entry offsets per chunk
};

__device__ __forceinline__ uint64_t be_u64(const uint8_t* p) {
  uint64_t v = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) v = (v << 8) | p[i];
  return v;
}
__device__ __forceinline__ uint32_t be_u32(const uint8_t* p) {
  return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | (uint32_t)p[3];
}

// kind of the element whose prefix is at p: 0 record, 1 watermark, 2 latency marker, -1 not an element
__device__ __forceinline__ int dec_kind(const DecSpec& d, uint32_t len, uint8_t tag) {
  if (tag == 0 && len == (uint32_t)d.rec_ts_len) return 0;
  if (tag == 1 && len == (uint32_t)d.rec_len) return 0;
  if (tag == 2 && len == 9u) return 1;
  if (tag == 3 && len == 17u) return 2;
  return -1;
}

// table entry per (chunk, candidate): alive | exit offset + 32768 (<< 1) | records (<< 17) | watermarks
// (<< 33) | latency markers (<< 49).  exit = where the chain leaves the chunk, relative to its end
// (negative: the stream ends inside an element that starts in this chunk)
__device__ __forceinline__ uint64_t dec_pack(bool alive, int exit, uint32_t nr, uint32_t nw, uint32_t nl) {
  return (alive ? 1ull : 0ull) | ((uint64_t)(exit + 32768) << 1) | ((uint64_t)nr << 17) | ((uint64_t)nw << 33) |
         ((uint64_t)nl << 49);
}
__device__ __forceinline__ bool dec_alive(uint64_t t) { return t & 1ull; }
__device__ __forceinline__ int dec_exit(uint64_t t) { return (int)((t >> 1) & 0xFFFF) - 32768; }

__global__ __launch_bounds__(DEC_THREADS) void k_dec_scan(DecSpec d, uint64_t* table, int32_t* conv) {
  __shared__ uint8_t buf[DEC_CHUNK + 8];
  __shared__ int32_t agree;   // the common exit of the surviving chains; INT32_MIN: none survived; INT32_MAX: differ
  const int64_t c = blockIdx.x;
  const int64_t start = c * DEC_CHUNK;
  const int clen = (int)min<int64_t>(DEC_CHUNK, d.nbytes - start);
  const int slen = (int)min<int64_t>(DEC_CHUNK + 8, d.nbytes - start);
  for (int i = threadIdx.x; i < slen; i += DEC_THREADS) buf[i] = d.bytes[start + i];
  if (threadIdx.x == 0) agree = INT32_MIN;
  __syncthreads();
  const int e = threadIdx.x;
  if (e < d.maxe) {
    int pos = e;
    bool alive = e < clen;   // a true entry lies inside the chunk (an element cut by the end ends the chain before)
    uint32_t nr = 0, nw = 0, nl = 0;
    int exit = 0;
    while (alive && pos < clen) {
      if (pos + 5 > slen) { exit = pos - clen; break; }          // prefix + tag beyond the stream's end
      const uint32_t len = be_u32(buf + pos);
      const int k = dec_kind(d, len, buf[pos + 4]);
      if (k < 0) { alive = false; break; }
      if (start + pos + 4 + (int64_t)len > d.nbytes) { exit = pos - clen; break; }   // cut by the end
      nr += k == 0; nw += k == 1; nl += k == 2;
      pos += 4 + (int)len;
      exit = pos - clen;
    }
    if (alive && pos >= clen) exit = pos - clen;
    table[c * d.maxe + e] = dec_pack(alive, exit, nr, nw, nl);
    if (alive) {
      const int cur = atomicCAS(&agree, INT32_MIN, exit);
      if (cur != INT32_MIN && cur != exit) atomicExch(&agree, INT32_MAX);
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) conv[c] = agree;
}

// entry offset of every chunk (the stream starts at an element boundary), then the exclusive prefix of
// each chunk's records / watermarks / latency markers.  One workgroup.
constexpr int DEC_LINK_THREADS = 1024;
__global__ __launch_bounds__(DEC_LINK_THREADS) void k_dec_link(DecSpec d, const uint64_t* table, const int32_t* conv,
                                                              int32_t* entry, int64_t* base, int64_t* totals,
                                                              int64_t* unknown, int32_t* err) {
  __shared__ int64_t wsum[3][DEC_LINK_THREADS / 64];
  __shared__ int32_t nunk;
  const int NT = DEC_LINK_THREADS;
  const int64_t per = (d.nchunks + NT - 1) / NT;
  const int64_t c0 = (int64_t)threadIdx.x * per, c1 = min(c0 + per, d.nchunks);
  // entries known from the previous chunk's agreeing survivors
  int32_t unk = 0;
  for (int64_t c = c0; c < c1; ++c) {
    int32_t en;
    if (c == 0) en = 0;
    else {
      const int32_t a = conv[c - 1];
      // -3: corrupt, -2: resolve in order, -1: the stream ended inside the previous chunk's last element
      en = (a == INT32_MIN) ? -3 : (a == INT32_MAX) ? -2 : (a < 0 ? -1 : a);
    }
    entry[c] = en;
    unk += en == -2;
  }
  // the undecided chunks, in order, into one list
  int64_t u = unk;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  int64_t incl = u;
  for (int o = 1; o < 64; o <<= 1) { const int64_t y = __shfl_up(incl, o); if (lane >= o) incl += y; }
  if (lane == 63) wsum[0][wv] = incl;
  __syncthreads();
  int64_t off = incl - u;
  for (int w = 0; w < wv; ++w) off += wsum[0][w];
  if (threadIdx.x == NT - 1) nunk = (int32_t)(off + u);
  for (int64_t c = c0; c < c1; ++c) if (entry[c] == -2) unknown[off++] = c;
  __syncthreads();
  if (threadIdx.x == 0) {   // nearly always empty
    for (int32_t i = 0; i < nunk; ++i) {
      const int64_t c = unknown[i];
      const int32_t prev = entry[c - 1];
      if (prev < 0) { entry[c] = prev == -1 ? -1 : -3; continue; }
      const uint64_t t = table[(c - 1) * d.maxe + prev];
      entry[c] = !dec_alive(t) ? -3 : dec_exit(t) < 0 ? -1 : dec_exit(t);
    }
  }
  __syncthreads();
  // per chunk: its counts along the true chain (the chain past a cut element: the chunks after carry
  // nothing), then the exclusive prefix
  int64_t cnt[3] = {0, 0, 0};
  for (int64_t c = c0; c < c1; ++c) {
    const int32_t en = entry[c];
    if (en == -3 || (en >= 0 && !dec_alive(table[c * d.maxe + en]))) { atomicExch(err, 1); continue; }
    if (en < 0) continue;
    const uint64_t t = table[c * d.maxe + en];
    cnt[0] += (t >> 17) & 0xFFFF; cnt[1] += (t >> 33) & 0xFFFF; cnt[2] += (t >> 49) & 0x7FFF;
  }
  int64_t offs[3];
  for (int k = 0; k < 3; ++k) {
    int64_t in = cnt[k];
    for (int o = 1; o < 64; o <<= 1) { const int64_t y = __shfl_up(in, o); if (lane >= o) in += y; }
    __syncthreads();
    if (lane == 63) wsum[k][wv] = in;
    __syncthreads();
    offs[k] = in - cnt[k];
    for (int w = 0; w < wv; ++w) offs[k] += wsum[k][w];
    if (threadIdx.x == NT - 1) totals[k] = offs[k] + cnt[k];
  }
  for (int64_t c = c0; c < c1; ++c) {
    base[3 * c + 0] = offs[0]; base[3 * c + 1] = offs[1]; base[3 * c + 2] = offs[2];
    const int32_t en = entry[c];
    if (en < 0 || !dec_alive(table[c * d.maxe + en])) continue;
    const uint64_t t = table[c * d.maxe + en];
    offs[0] += (t >> 17) & 0xFFFF; offs[1] += (t >> 33) & 0xFFFF; offs[2] += (t >> 49) & 0x7FFF;
  }
  // bytes of whole elements: up to the last chunk's chain end
  if (threadIdx.x == 0) {
    int64_t consumed = 0;
    for (int64_t c = d.nchunks - 1; c >= 0; --c) {
      const int32_t en = entry[c];
      if (en < 0) continue;
      const uint64_t t = table[c * d.maxe + en];
      const int64_t clen = min<int64_t>(DEC_CHUNK, d.nbytes - c * DEC_CHUNK);
      consumed = c * DEC_CHUNK + clen + dec_exit(t);
      break;
    }
    totals[3] = consumed;
  }
}

struct DecOut {
  int64_t *key, *f1, *ts, *val, *wm, *wm_pos, *lm, *lm_pos;
  int32_t* key_hash;
  int64_t record_cap, marker_cap;
};

__global__ __launch_bounds__(DEC_THREADS) void k_dec_emit(DecSpec d, const int32_t* entry, const int64_t* base,
                                                         DecOut o, int32_t* err) {
  __shared__ uint8_t buf[DEC_CHUNK + DEC_MAXE + 8];
  __shared__ int16_t el_pos[DEC_MAXEL];     // element start (prefix) within the chunk
  __shared__ int16_t el_rank[DEC_MAXEL];    // index among the chunk's elements of its kind
  __shared__ int8_t el_kind[DEC_MAXEL];
  __shared__ int32_t nel;
  const int64_t c = blockIdx.x;
  const int32_t en = entry[c];
  if (en < 0) return;   // uniform: past the stream's last whole element
  const int64_t start = c * DEC_CHUNK;
  const int clen = (int)min<int64_t>(DEC_CHUNK, d.nbytes - start);
  const int slen = (int)min<int64_t>(DEC_CHUNK + DEC_MAXE + 8, d.nbytes - start);
  for (int i = threadIdx.x; i < slen; i += DEC_THREADS) buf[i] = d.bytes[start + i];
  __syncthreads();
  if (threadIdx.x == 0) {   // the chunk's true chain, once
    int pos = en, n = 0, r[3] = {0, 0, 0};
    while (pos < clen && pos + 5 <= slen && n < DEC_MAXEL) {
      const uint32_t len = be_u32(buf + pos);
      const int k = dec_kind(d, len, buf[pos + 4]);
      if (k < 0) { atomicExch(err, 1); break; }
      if (start + pos + 4 + (int64_t)len > d.nbytes) break;   // cut by the end: the next call's
      el_pos[n] = (int16_t)pos; el_kind[n] = (int8_t)k; el_rank[n] = (int16_t)r[k]++;
      ++n;
      pos += 4 + (int)len;
    }
    nel = n;
  }
  __syncthreads();
  for (int i = threadIdx.x; i < nel; i += DEC_THREADS) {
    const uint8_t* p = buf + el_pos[i] + 4;   // the tag
    const int k = el_kind[i];
    if (k == 0) {
      const int64_t j = base[3 * c] + el_rank[i];
      if (j >= o.record_cap) { atomicExch(err, 2); continue; }
      const bool has_ts = p[0] == 0;
      const int64_t ts = has_ts ? (int64_t)be_u64(p + 1) : INT64_MIN;
      const uint8_t* t = p + (has_ts ? 9 : 1);
      const int64_t key = d.key_int ? (int64_t)(int32_t)be_u32(t + d.key_off) : (int64_t)be_u64(t + d.key_off);
      o.key[j] = key;
      if (o.key_hash) o.key_hash[j] = (int32_t)key;   // Integer.hashCode
      o.ts[j] = ts;
      o.f1[j] = d.f1_off < 0 ? ts : d.f1_int ? (int64_t)(int32_t)be_u32(t + d.f1_off) : (int64_t)be_u64(t + d.f1_off);
      o.val[j] = (int64_t)be_u64(t + d.val_off);
    } else {
      const int64_t j = base[3 * c + k] + el_rank[i];
      // position: the records before it (this chunk's before element i, found backwards: markers are rare)
      int32_t before = 0;
      for (int q = i - 1; q >= 0; --q) if (el_kind[q] == 0) { before = el_rank[q] + 1; break; }
      const int64_t rpos = base[3 * c] + before;
      if (j >= o.marker_cap) { atomicExch(err, 2); continue; }
      if (k == 1) {
        o.wm[j] = (int64_t)be_u64(p + 1);
        o.wm_pos[j] = rpos;
      } else {   // latency marker: markedTime, then vertexId << 32 | subtaskIndex
        o.lm[2 * j] = (int64_t)be_u64(p + 1);
        o.lm[2 * j + 1] = (int64_t)(((uint64_t)be_u32(p + 9) << 32) | be_u32(p + 13));
        o.lm_pos[j] = rpos;
      }
    }
  }
}

}  // namespace fw

int fw_decode(fw_engine* e, const fw_tuple_schema* sc, const void* bytes, int64_t nbytes, int32_t mem, int64_t* key,
              int32_t* key_hash, int64_t* f1, int64_t* ts, void* value, int64_t record_cap, int64_t* wm,
              int64_t* wm_pos, int64_t* lm, int64_t* lm_pos, int64_t marker_cap, fw_decode_counts* out) {
  using namespace fw;
  if (!e || !sc || !out || (nbytes > 0 && !bytes) || nbytes < 0) return FW_ERR_INVALID_ARG;
  if (e->sticky) return e->sticky;
  std::memset(out, 0, sizeof(*out));
  if (sc->n_fields < 1 || sc->n_fields > FW_DECODE_MAX_FIELDS || sc->key_field < 0 || sc->key_field >= sc->n_fields ||
      sc->value_field < 0 || sc->value_field >= sc->n_fields || sc->f1_field < -1 || sc->f1_field >= sc->n_fields)
    return reject(e, FW_ERR_INVALID_ARG, "bad tuple schema");
  DecSpec d{};
  int off = 0;
  d.f1_off = -1;
  for (int i = 0; i < sc->n_fields; ++i) {
    const int t = sc->field_type[i];
    if (t != FW_FT_LONG && t != FW_FT_DOUBLE && t != FW_FT_INT) return reject(e, FW_ERR_UNSUPPORTED, "field type");
    if (i == sc->key_field) {
      if (t == FW_FT_DOUBLE) return reject(e, FW_ERR_UNSUPPORTED, "double key");
      d.key_off = off; d.key_int = t == FW_FT_INT;
    }
    if (i == sc->f1_field) {
      if (t == FW_FT_DOUBLE) return reject(e, FW_ERR_UNSUPPORTED, "double f1");
      d.f1_off = off; d.f1_int = t == FW_FT_INT;
    }
    if (i == sc->value_field) {
      const int want = e->s.vt == FW_VALUE_F64 ? FW_FT_DOUBLE : FW_FT_LONG;
      if (t != want) return reject(e, FW_ERR_UNSUPPORTED, "value field type differs from the engine's value type");
      d.val_off = off;
    }
    off += t == FW_FT_INT ? 4 : 8;
  }
  if (d.key_int && !key_hash) return reject(e, FW_ERR_INVALID_ARG, "an int key needs the key_hash column");
  d.rec_len = 1 + off;
  d.rec_ts_len = 9 + off;
  d.maxe = 4 + std::max(d.rec_ts_len, 17);
  d.nbytes = nbytes;
  d.nchunks = (nbytes + DEC_CHUNK - 1) / DEC_CHUNK;
  if (nbytes == 0) return FW_OK;
  HIPCHK(e, hipSetDevice(e->dev));
  // grow-only scratch
  auto grow = [&](void*& p, size_t& cap, size_t need) -> hipError_t {
    if (cap >= need) return hipSuccess;
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
    hipError_t r = hipMalloc(&p, need);
    if (r == hipSuccess) cap = need;
    return r;
  };
  const size_t nc = (size_t)d.nchunks;
  HIPCHK(e, grow(e->dec_table, e->dec_table_cap, nc * (size_t)d.maxe * 8));
  HIPCHK(e, grow(e->dec_small, e->dec_small_cap, nc * (4 + 4 + 8 + 24) + 64));
  const uint8_t* src = (const uint8_t*)bytes;
  if (mem == FW_MEM_HOST) {
    HIPCHK(e, grow(e->dec_bytes, e->dec_bytes_cap, (size_t)nbytes));
    HIPCHK(e, hipMemcpyAsync(e->dec_bytes, bytes, (size_t)nbytes, hipMemcpyHostToDevice, e->stream));
    src = (const uint8_t*)e->dec_bytes;
  }
  d.bytes = src;
  uint8_t* sm = (uint8_t*)e->dec_small;
  int32_t* conv = (int32_t*)sm;
  int32_t* entry = conv + nc;
  int64_t* unknown = (int64_t*)(((uintptr_t)(entry + nc) + 7) & ~(uintptr_t)7);
  int64_t* base = unknown + nc;
  int64_t* totals = base + 3 * nc;   // [4] records, watermarks, latency markers, consumed bytes
  int32_t* err = (int32_t*)(totals + 4);
  HIPCHK(e, hipMemsetAsync(err, 0, 4, e->stream));
  uint64_t* table = (uint64_t*)e->dec_table;
  hipLaunchKernelGGL(k_dec_scan, dim3((unsigned)nc), dim3(DEC_THREADS), 0, e->stream, d, table, conv);
  hipLaunchKernelGGL(k_dec_link, dim3(1), dim3(DEC_LINK_THREADS), 0, e->stream, d, table, conv, entry, base, totals,
                     unknown, err);
  DecOut o{key, f1, ts, (int64_t*)value, wm, wm_pos, lm, lm_pos, key_hash, record_cap, marker_cap};
  hipLaunchKernelGGL(k_dec_emit, dim3((unsigned)nc), dim3(DEC_THREADS), 0, e->stream, d, entry, base, o, err);
  HIPCHK(e, hipGetLastError());
  int64_t tot[4];
  int32_t herr = 0;
  HIPCHK(e, hipMemcpyAsync(tot, totals, sizeof(tot), hipMemcpyDeviceToHost, e->stream));
  HIPCHK(e, hipMemcpyAsync(&herr, err, 4, hipMemcpyDeviceToHost, e->stream));
  HIPCHK(e, hipStreamSynchronize(e->stream));
  if (herr == 1) return reject(e, FW_ERR_INVALID_ARG, "corrupt stream: no element chain through the bytes");
  out->n_records = tot[0];
  out->n_watermarks = tot[1];
  out->n_latency_markers = tot[2];
  out->consumed = tot[3];
  if (herr == 2 || tot[0] > record_cap || tot[1] > marker_cap || tot[2] > marker_cap)
    return reject(e, FW_ERR_CAPACITY, "decode output capacity exceeded");
  return FW_OK;
}
