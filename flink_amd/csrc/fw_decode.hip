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
// SpillingAdaptiveSpanningRecordDeserializer).  Here the bytes are cut into 512-byte chunks; for every chunk
// one lane follows the length chain from each offset an element could start at (elements are shorter than
// DEC_MAXE bytes), validating every step against the lengths and tags the schema allows.  Chains from
// different offsets merge within a few elements and the ones off the boundaries die at a bad length or
// tag, so the surviving chains of a chunk nearly always leave it at one offset: the next chunk's entry,
// known without the chunks before.  The rare chunks whose survivors disagree are linked one after
// another.  Then each chunk's true chain is walked twice more, once to count its records and markers
// (an exclusive scan places them) and once to decode them.  One lane per chunk throughout: a chain is a
// sequence of dependent steps, so a wave keeps 64 chains going (one chunk per workgroup, walked by one
// lane, left the other 63 idle and cost ~1 ms per 4 Mi records).
#pragma once

namespace fw {

constexpr int DEC_CHUNK = 512;     // bytes per chunk
constexpr int DEC_MAXE = 4 + 1 + 8 + 8 * FW_DECODE_MAX_FIELDS;   // longest element with its length prefix
constexpr int DEC_T = 64;          // chunks per workgroup, one lane of wave 0 each: the workgroup's chunks are
                                   // staged in LDS with 16-B loads (a lane walking its chunk in global memory
                                   // issued one uncoalesced byte load per field byte: ~1 line request per lane-byte)
constexpr int DEC_TW = 256;        // threads per workgroup: all stage the chunks (one round of loads) and decode
constexpr int DEC_SPILL = 68;      // bytes after a chunk an element starting in it can reach (>= DEC_MAXE)
constexpr int DEC_STRIDE = DEC_CHUNK + DEC_SPILL;   // LDS bytes per chunk: 145 words apart (odd), so the 64
                                   // lanes reading the same offset of their chunks hit 64 different banks
constexpr int DEC_LDS = DEC_T * DEC_STRIDE;
constexpr int DEC_SCAN = 1024;     // chunks per level-1 scan block

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
// the same from 4-byte aligned LDS words: two (three) word reads and byte alignment instead of 4 (8) byte reads
__device__ __forceinline__ uint32_t lds_be_u32(const uint8_t* p) {
  const uint32_t a = (uint32_t)(uintptr_t)p & 3u;
  const uint32_t* w = (const uint32_t*)(p - a);
  const uint32_t x = __builtin_amdgcn_alignbyte(w[1], w[0], a);
  return __builtin_bswap32(x);
}
__device__ __forceinline__ uint64_t lds_be_u64(const uint8_t* p) {
  const uint32_t a = (uint32_t)(uintptr_t)p & 3u;
  const uint32_t* w = (const uint32_t*)(p - a);
  const uint32_t w0 = w[0], w1 = w[1], w2 = w[2];
  const uint32_t lo = __builtin_amdgcn_alignbyte(w1, w0, a), hi = __builtin_amdgcn_alignbyte(w2, w1, a);
  return ((uint64_t)__builtin_bswap32(lo) << 32) | (uint64_t)__builtin_bswap32(hi);
}

// kind of the element with length len and tag: 0 record, 1 watermark, 2 latency marker, -1 not an element
__device__ __forceinline__ int dec_kind(const DecSpec& d, uint32_t len, uint8_t tag) {
  if (tag == 0 && len == (uint32_t)d.rec_ts_len) return 0;
  if (tag == 1 && len == (uint32_t)d.rec_len) return 0;
  if (tag == 2 && len == 9u) return 1;
  if (tag == 3 && len == 17u) return 2;
  return -1;
}

// the chain from offset e of chunk c: DEC_DEAD (a step that is no element), or where it leaves the chunk
// relative to the chunk's end (negative: the stream ends inside an element starting in this chunk)
constexpr int DEC_DEAD = INT32_MIN;
struct DecChunk {
  const uint8_t* b;   // the chunk's first byte (in LDS)
  int clen;           // its bytes
  int rem;            // bytes of the stream from its first byte on (capped at 2^30: every test is within a chunk + spill)
};
// the workgroup's DEC_T chunks into LDS, each at DEC_STRIDE with its own copy of the DEC_SPILL bytes after it
// (the next chunk's first ones), then this lane's chunk.  Global loads of 16 B, LDS stores of 4 B
// the 16 bytes at group offset q (a multiple of 16: they lie in one chunk), and again after the previous chunk
// when they are among the first DEC_SPILL bytes of theirs; one address per copy, four word stores
__device__ __forceinline__ void dec_put16(uint8_t* buf, int q, const uint4& v) {
  const int i = q >> 9, o = q & (DEC_CHUNK - 1);
  static_assert(DEC_CHUNK == 512 && DEC_SPILL % 4 == 0, "chunk layout");
  if (i < DEC_T) {
    uint32_t* d = (uint32_t*)(buf + i * DEC_STRIDE + o);
    d[0] = v.x; d[1] = v.y; d[2] = v.z; d[3] = v.w;
  }
  if (i > 0 && o < DEC_SPILL) {   // (the spill copy ends at DEC_SPILL: the next chunk's copy follows it)
    uint32_t* d = (uint32_t*)(buf + (i - 1) * DEC_STRIDE + DEC_CHUNK + o);
    d[0] = v.x;
    if (o + 4 < DEC_SPILL) d[1] = v.y;
    if (o + 8 < DEC_SPILL) d[2] = v.z;
    if (o + 12 < DEC_SPILL) d[3] = v.w;
  }
}
__device__ __forceinline__ void dec_put1(uint8_t* buf, int q, uint8_t b) {
  const int i = q / DEC_CHUNK, o = q % DEC_CHUNK;
  if (i < DEC_T) buf[i * DEC_STRIDE + o] = b;
  if (i > 0 && o < DEC_SPILL) buf[(i - 1) * DEC_STRIDE + DEC_CHUNK + o] = b;
}
// the DEC_T chunks from chunk c0 on into LDS, then this lane's chunk
__device__ __forceinline__ DecChunk dec_stage_at(const DecSpec& d, uint8_t* buf, int64_t c0) {
  const int64_t g0 = c0 * DEC_CHUNK;
  const int len = (int)min<int64_t>(DEC_T * DEC_CHUNK + DEC_SPILL, d.nbytes - g0);
  const uint8_t* src = d.bytes + g0;
  int done = 0;
  if (((uintptr_t)src & 15) == 0) {
    const int nv = len >> 4;
    constexpr int NU = (DEC_T * DEC_CHUNK + DEC_SPILL + 16 * DEC_TW - 1) / (16 * DEC_TW);   // one round of loads
    for (int i0 = 0; i0 < nv; i0 += NU * DEC_TW) {
      uint4 v[NU];
#pragma unroll
      for (int u = 0; u < NU; ++u) { const int i = i0 + u * DEC_TW + (int)threadIdx.x; if (i < nv) v[u] = ((const uint4*)src)[i]; }
#pragma unroll
      for (int u = 0; u < NU; ++u) {
        const int i = i0 + u * DEC_TW + (int)threadIdx.x;
        if (i < nv) dec_put16(buf, 16 * i, v[u]);
      }
    }
    done = nv << 4;
  }
  for (int i = done + (int)threadIdx.x; i < len; i += DEC_TW) dec_put1(buf, i, src[i]);
  __syncthreads();
  const int lane = (int)threadIdx.x & (DEC_T - 1);
  const int64_t c = c0 + lane;
  const int64_t start = c * DEC_CHUNK;
  return {buf + lane * DEC_STRIDE, (int)max<int64_t>(0, min<int64_t>(DEC_CHUNK, d.nbytes - start)),
          (int)min<int64_t>(d.nbytes - start, (int64_t)1 << 30)};
}
__device__ __forceinline__ DecChunk dec_stage_group(const DecSpec& d, uint8_t* buf) {
  return dec_stage_at(d, buf, (int64_t)blockIdx.x * DEC_T);
}
// the element header at LDS position p (4-byte BE length, then the tag) from two aligned word reads
__device__ __forceinline__ void dec_header(const uint8_t* p, uint32_t& len, uint32_t& tag) {
  const uint32_t a = (uint32_t)(uintptr_t)p & 3u;
  const uint32_t* w = (const uint32_t*)(p - a);
  const uint32_t w0 = w[0], w1 = w[1];
  len = __builtin_bswap32(__builtin_amdgcn_alignbyte(w1, w0, a));
  tag = (w1 >> (8 * a)) & 0xffu;
}
// after a record of length len with tag at pos - (4 + len): how many of the next DEC_FF elements are records of
// the same length and tag, complete in the stream and starting in the chunk.  The positions are known in
// advance, so the DEC_FF header reads are independent (one LDS round trip instead of DEC_FF dependent steps):
// a run of same-shape records is the common stream, markers and the chunk's end break it
constexpr int DEC_FF = 8;
__device__ __forceinline__ int dec_ff(const DecChunk& ch, int pos, uint32_t len, uint32_t tag) {
  const int L = 4 + (int)len;
  int m = 0;
  bool ok = true;
#pragma unroll
  for (int j = 0; j < DEC_FF; ++j) {
    const int p = pos + j * L;
    const bool in = p < ch.clen && p + L <= ch.rem;
    uint32_t hl = 0, ht = 0;
    dec_header(ch.b + (in ? p : 0), hl, ht);
    ok = ok && in && hl == len && ht == tag;
    m += ok;
  }
  return m;
}
template <typename F>
__device__ __forceinline__ int dec_walk(const DecSpec& d, const DecChunk& ch, int e, F&& on_element) {
  int pos = e;
  while (pos < ch.clen) {
    if (pos + 5 > ch.rem) return pos - ch.clen;                       // prefix + tag beyond the stream's end
    uint32_t len, tag;
    dec_header(ch.b + pos, len, tag);
    const int k = dec_kind(d, len, (uint8_t)tag);
    if (k < 0) return DEC_DEAD;
    if (pos + 4 + (int)len > ch.rem) return pos - ch.clen;            // cut by the end: the next call's
    on_element(pos, k);
    pos += 4 + (int)len;
    if (k == 0) {
      const int m = dec_ff(ch, pos, len, tag);
      for (int j = 0; j < m; ++j) on_element(pos + j * (4 + (int)len), 0);
      pos += m * (4 + (int)len);
    }
  }
  return pos - ch.clen;
}

// a candidate chain's outcome in one word: its exit (biased by DEC_XB) and the records, watermarks and latency
// markers along it (a 512-byte chunk holds at most 39 elements: 6 bits each)
constexpr int DEC_XB = 512;
__device__ __forceinline__ int32_t dec_cpack(int x, int n0, int n1, int n2) {
  return (x + DEC_XB) | (n0 << 10) | (n1 << 16) | (n2 << 22);
}
__device__ __forceinline__ int dec_cexit(int32_t v) { return (v & 1023) - DEC_XB; }
constexpr int DEC_W = DEC_TW / 64;       // waves per workgroup: each takes every DEC_W-th candidate of every chunk
constexpr int DEC_SW = 2;                // survivors kept per wave and chunk (entry offset << 32 | outcome)
constexpr int DEC_S = DEC_W * DEC_SW;    // ... per chunk; beyond them a chunk's count is walked again
__device__ __forceinline__ int32_t dec_agree(int32_t a, int32_t x) {
  return a == INT32_MIN ? x : (x == INT32_MIN || a == x) ? a : INT32_MAX;
}

// the bytes of group g (DEC_T chunks + the spill after them) in registers: 16-B loads, one round; *ok false when
// they cannot be loaded that way (an unaligned source): the group is then staged byte by byte
constexpr int DEC_NU = (DEC_T * DEC_CHUNK + DEC_SPILL + 16 * DEC_TW - 1) / (16 * DEC_TW);
__device__ __forceinline__ void dec_prefetch(const DecSpec& d, int64_t g, uint4 (&v)[DEC_NU]) {
  const int64_t g0 = g * DEC_T * DEC_CHUNK;
  const int len = (int)min<int64_t>(DEC_T * DEC_CHUNK + DEC_SPILL, d.nbytes - g0);
  const uint4* src = (const uint4*)(d.bytes + g0);
  const int nv = len >> 4;
#pragma unroll
  for (int u = 0; u < DEC_NU; ++u) {
    const int i = u * DEC_TW + (int)threadIdx.x;
    if (i < nv) v[u] = src[i];
  }
}
// group g into LDS from the prefetched registers (+ the bytes after the last whole 16-B unit); then this lane's chunk
__device__ __forceinline__ DecChunk dec_stage_regs(const DecSpec& d, uint8_t* buf, int64_t g, const uint4 (&v)[DEC_NU]) {
  const int64_t g0 = g * DEC_T * DEC_CHUNK;
  const int len = (int)min<int64_t>(DEC_T * DEC_CHUNK + DEC_SPILL, d.nbytes - g0);
  const int nv = len >> 4;
#pragma unroll
  for (int u = 0; u < DEC_NU; ++u) {
    const int i = u * DEC_TW + (int)threadIdx.x;
    if (i < nv) dec_put16(buf, 16 * i, v[u]);
  }
  for (int i = (nv << 4) + (int)threadIdx.x; i < len; i += DEC_TW) dec_put1(buf, i, d.bytes[g0 + i]);
  __syncthreads();
  const int lane = (int)threadIdx.x & (DEC_T - 1);
  const int64_t start = (g * DEC_T + lane) * DEC_CHUNK;
  return {buf + lane * DEC_STRIDE, (int)max<int64_t>(0, min<int64_t>(DEC_CHUNK, d.nbytes - start)),
          (int)min<int64_t>(d.nbytes - start, (int64_t)1 << 30)};
}

// per chunk and wave: the exit its surviving candidate chains agree on (INT32_MIN: none survived, INT32_MAX: they
// differ) and up to DEC_SW survivors with their counts, so the true chain's counts are known once its entry is
// (no second walk).  The workgroup's waves share a chunk's candidates (wave w takes e = w, w + DEC_W, ...; lane =
// chunk), so DEC_W chains per chunk run at once; each wave writes its own results (no LDS beyond the chunks)
__global__ __launch_bounds__(DEC_TW) void k_dec_scan(DecSpec d, int32_t* conv, int64_t* surv, int32_t* nsurv,
                                                    int32_t* err, int64_t ngroups) {
  __shared__ __attribute__((aligned(16))) uint8_t buf[DEC_LDS];
  if (blockIdx.x == 0 && threadIdx.x == 0) *err = 0;   // (read by the kernels after this one)
  // persistent: groups g = blockIdx.x, + gridDim.x, ..., the next group's bytes loading into registers while this
  // one's candidates are walked (a 16-B aligned source; otherwise each group is staged as it comes)
  const bool aligned = ((uintptr_t)d.bytes & 15) == 0;
  uint4 v[DEC_NU];
  if (aligned && (int64_t)blockIdx.x < ngroups) dec_prefetch(d, blockIdx.x, v);
  for (int64_t g = blockIdx.x; g < ngroups; g += gridDim.x) {
  __syncthreads();   // the previous group's LDS is read
  const DecChunk ch = aligned ? dec_stage_regs(d, buf, g, v) : dec_stage_at(d, buf, g * DEC_T);
  if (aligned && g + gridDim.x < ngroups) dec_prefetch(d, g + gridDim.x, v);
  const int lane = (int)threadIdx.x & (DEC_T - 1), wv = (int)threadIdx.x >> 6;
  const int64_t c = g * DEC_T + lane;
  if (c >= d.nchunks) continue;
  const int lim = min(d.maxe, ch.clen);
  int32_t agree = INT32_MIN;
  int ns = 0;
  int64_t* sv = surv + c * DEC_S + wv * DEC_SW;
  // first the candidates' first headers, all at once (independent reads, no divergence): most offsets are no
  // element start and drop out here; a bit per candidate that can start a chain (or meets the stream's end)
  uint32_t live = 0;
  for (int i = 0, e = wv; e < lim; ++i, e += DEC_W) {
    bool ok = e + 5 > ch.rem;
    if (!ok) {
      uint32_t len, tag;
      dec_header(ch.b + e, len, tag);
      ok = dec_kind(d, len, (uint8_t)tag) >= 0;
    }
    live |= (ok ? 1u : 0u) << i;
  }
  // then the live candidates' chains, one step per iteration of a single loop whatever candidate it belongs to
  // (nested loops cost ~10x the steps)
  int e = live ? wv + DEC_W * (__ffs(live) - 1) : lim, pos = e, n0 = 0, n1 = 0, n2 = 0;
  live &= live - 1;
  while (e < lim) {
    int x = DEC_DEAD;
    bool fin = true;
    if (pos >= ch.clen || pos + 5 > ch.rem) {
      x = pos - ch.clen;
    } else {
      uint32_t len, tag;
      dec_header(ch.b + pos, len, tag);
      const int k = dec_kind(d, len, (uint8_t)tag);
      if (k < 0) x = DEC_DEAD;
      else if (pos + 4 + (int)len > ch.rem) x = pos - ch.clen;
      else {
        pos += 4 + (int)len;
        n0 += k == 0; n1 += k == 1; n2 += k == 2;
        if (k == 0) {
          const int m = dec_ff(ch, pos, len, tag);
          pos += m * (4 + (int)len);
          n0 += m;
        }
        fin = false;
      }
    }
    if (fin) {
      if (x != DEC_DEAD) {
        agree = dec_agree(agree, x);
        if (ns < DEC_SW) sv[ns] = ((int64_t)e << 32) | (uint32_t)dec_cpack(x, n0, n1, n2);
        ++ns;
      }
      e = live ? wv + DEC_W * (__ffs(live) - 1) : lim;
      live &= live - 1;
      pos = e;
      n0 = n1 = n2 = 0;
    }
  }
  conv[c * DEC_W + wv] = agree;
  nsurv[c * DEC_W + wv] = ns;
  }
}

// chunk c's chain from pos in global memory (the rare paths): its exit or DEC_DEAD, and its counts
__device__ __forceinline__ int32_t dec_walk_global(const DecSpec& d, int64_t c, int pos, int64_t n[3]) {
  const int64_t start = c * DEC_CHUNK;
  const int clen = (int)min<int64_t>(DEC_CHUNK, d.nbytes - start);
  const int64_t rem = d.nbytes - start;
  const uint8_t* b = d.bytes + start;
  n[0] = n[1] = n[2] = 0;
  while (true) {
    if (pos >= clen || pos + 5 > rem) return pos - clen;
    const uint32_t len = be_u32(b + pos);
    const int k = dec_kind(d, len, b[pos + 4]);
    if (k < 0) return DEC_DEAD;
    if (pos + 4 + (int64_t)len > rem) return pos - clen;
    n[k]++;
    pos += 4 + (int)len;
  }
}
// the entry a chunk's predecessor's survivors agree on (-2: they differ, -3: none survived: corrupt, -1: the
// stream ended inside the predecessor's last element)
__device__ __forceinline__ int32_t dec_agreed_entry(const int32_t* conv, int64_t c) {
  if (c == 0) return 0;
  int32_t a = INT32_MIN;
  for (int w = 0; w < DEC_W; ++w) a = dec_agree(a, conv[(c - 1) * DEC_W + w]);
  return (a == INT32_MIN) ? -3 : (a == INT32_MAX) ? -2 : (a < 0 ? -1 : a);
}

// per chunk: its entry (from its predecessor's agreeing survivors; where they differ — rare — from the last
// chunk whose entry they fix, walking the chunks after it in global memory), its counts along its true chain
// (from its survivors, else walked), then the exclusive prefix of the counts within blocks of DEC_SCAN chunks
// (base) and the block totals (btot)
__global__ __launch_bounds__(DEC_SCAN) void k_dec_bscan(DecSpec d, const int32_t* conv, const int64_t* surv,
                                                       const int32_t* nsurv, int32_t* entry, int32_t* cexit,
                                                       int64_t* base, int64_t* btot, int32_t* err) {
  __shared__ int64_t ws[3][DEC_SCAN / 64];
  const int64_t c = (int64_t)blockIdx.x * DEC_SCAN + threadIdx.x;
  int64_t v[3] = {0, 0, 0};
  if (c < d.nchunks) {
    int32_t en = dec_agreed_entry(conv, c);
    if (en == -2) {
      int64_t j = c - 1;
      int32_t ej = dec_agreed_entry(conv, j);
      while (ej == -2) ej = dec_agreed_entry(conv, --j);
      for (; j < c && ej >= 0; ++j) {   // entry of j known: its chain's exit is the entry of j + 1
        int64_t n[3];
        const int32_t x = dec_walk_global(d, j, ej, n);
        ej = x == DEC_DEAD ? -3 : x < 0 ? -1 : x;
      }
      en = ej;
    }
    int32_t x = DEC_DEAD;
    if (en == -3) atomicExch(err, 1);
    if (en >= 0) {
      const int clen = (int)min<int64_t>(DEC_CHUNK, d.nbytes - c * DEC_CHUNK);
      bool found = false;
      if (en >= clen) {   // the previous element covers the (last, short) chunk
        x = en - clen;
        found = true;
      } else {
        const int w = en % DEC_W;   // the wave that walked candidate en
        const int ns = min(nsurv[c * DEC_W + w], DEC_SW);
        for (int i = 0; i < ns && !found; ++i) {
          const int64_t sv = surv[c * DEC_S + w * DEC_SW + i];
          if ((int32_t)(sv >> 32) != en) continue;
          const int32_t pk = (int32_t)(uint32_t)sv;
          v[0] = (pk >> 10) & 63; v[1] = (pk >> 16) & 63; v[2] = (pk >> 22) & 63;
          x = dec_cexit(pk);
          found = true;
        }
      }
      if (!found) {   // not among the kept survivors (the wave found more): walked again
        x = dec_walk_global(d, c, en, v);
        if (x == DEC_DEAD) { atomicExch(err, 1); v[0] = v[1] = v[2] = 0; }
      }
    }
    entry[c] = en;
    cexit[c] = x;
  }
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    int64_t in = v[k];
    for (int o = 1; o < 64; o <<= 1) { const int64_t y = __shfl_up(in, o); if (lane >= o) in += y; }
    if (lane == 63) ws[k][wv] = in;
    v[k] = in - v[k];   // exclusive within the wave
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    int64_t off = 0, tot = 0;
    for (int w = 0; w < DEC_SCAN / 64; ++w) { off += w < wv ? ws[k][w] : 0; tot += ws[k][w]; }
    if (c < d.nchunks) base[3 * c + k] = v[k] + off;
    if (threadIdx.x == 0) btot[3 * blockIdx.x + k] = tot;
  }
}

// level 2: the blocks' exclusive offsets (in place), the totals and the bytes of whole elements.  One workgroup
__global__ __launch_bounds__(DEC_SCAN) void k_dec_top(DecSpec d, const int32_t* entry, const int32_t* cexit, int64_t* btot,
                                                     int64_t nblk, int64_t* totals) {
  __shared__ int64_t ws[3][DEC_SCAN / 64];
  const int64_t per = (nblk + DEC_SCAN - 1) / DEC_SCAN;
  const int64_t b0 = (int64_t)threadIdx.x * per, b1 = min(b0 + per, nblk);
  int64_t sum[3] = {0, 0, 0};
  for (int64_t b = b0; b < b1; ++b) for (int k = 0; k < 3; ++k) sum[k] += btot[3 * b + k];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  int64_t ex[3];
  for (int k = 0; k < 3; ++k) {
    int64_t in = sum[k];
    for (int o = 1; o < 64; o <<= 1) { const int64_t y = __shfl_up(in, o); if (lane >= o) in += y; }
    if (lane == 63) ws[k][wv] = in;
    ex[k] = in - sum[k];
  }
  __syncthreads();
  for (int k = 0; k < 3; ++k) {
    int64_t off = 0, tot = 0;
    for (int w = 0; w < DEC_SCAN / 64; ++w) { off += w < wv ? ws[k][w] : 0; tot += ws[k][w]; }
    ex[k] += off;
    if (threadIdx.x == 0) totals[k] = tot;
  }
  for (int64_t b = b0; b < b1; ++b)
    for (int k = 0; k < 3; ++k) { const int64_t t = btot[3 * b + k]; btot[3 * b + k] = ex[k]; ex[k] += t; }
  // bytes of whole elements: up to the last chunk's chain end
  if (threadIdx.x == 0) {
    int64_t consumed = 0;
    for (int64_t c = d.nchunks - 1; c >= 0; --c) {
      if (entry[c] < 0 || cexit[c] == DEC_DEAD) continue;
      const int64_t clen = min<int64_t>(DEC_CHUNK, d.nbytes - c * DEC_CHUNK);
      consumed = c * DEC_CHUNK + clen + cexit[c];
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

// records of a workgroup's chunks, at most: a record element is 4 + rec_len bytes or more (the list is sized per
// schema in dynamic LDS, so a workgroup fits four to a CU: 37 KB of chunks + ~2.3 KB for Tuple3 records)
__host__ __device__ inline int dec_maxrec(int rec_len) { return DEC_T * (DEC_CHUNK / (4 + rec_len) + 1); }
// each chunk's true chain once more: every lane lists its records' LDS positions at their rank within the
// workgroup (its chunks' records are one contiguous run of the output), and the workgroup then decodes them
// in rank order, so the column stores are coalesced; markers (rare) are written by their lane.  Persistent: a
// workgroup takes groups g = blockIdx.x, + gridDim.x, ..., the next group's bytes loading into registers while
// this one is walked and decoded (a 16-B aligned source; otherwise each group is staged as it comes)
__global__ __launch_bounds__(DEC_TW) void k_dec_emit(DecSpec d, const int32_t* entry, const int64_t* base_in,
                                                   const int64_t* btop, DecOut o, int32_t* err, const int64_t* totals,
                                                   unsigned int* done, int64_t* host_counts, int64_t ngroups) {
  __shared__ __attribute__((aligned(16))) uint8_t buf[DEC_LDS];
  extern __shared__ uint16_t rpos[];       // [dec_maxrec(d.rec_len)] LDS position of each record's tag
  const int maxrec = dec_maxrec(d.rec_len);
  __shared__ int64_t r0_s;
  __shared__ int32_t nrec_s;
  const bool aligned = ((uintptr_t)d.bytes & 15) == 0;
  uint4 v[DEC_NU];
  if (aligned && (int64_t)blockIdx.x < ngroups) dec_prefetch(d, blockIdx.x, v);
  for (int64_t g = blockIdx.x; g < ngroups; g += gridDim.x) {
    __syncthreads();   // the previous group's LDS is read
    const DecChunk ch = aligned ? dec_stage_regs(d, buf, g, v) : dec_stage_at(d, buf, g * DEC_T);
    if (aligned && g + gridDim.x < ngroups) dec_prefetch(d, g + gridDim.x, v);   // in flight during the work below
    const int64_t c = g * DEC_T + threadIdx.x;
    const int64_t cfirst = g * DEC_T;
    const int64_t bfirst = cfirst / DEC_SCAN;
    if (threadIdx.x == 0) { r0_s = btop[3 * bfirst] + base_in[3 * cfirst]; nrec_s = 0; }
    __syncthreads();
    const int32_t en = (threadIdx.x < DEC_T && c < d.nchunks) ? entry[c] : -1;
    int32_t nr = 0;
    if (en >= 0) {   // past the stream's last whole element (or corrupt: reported by k_dec_bscan) otherwise
      const int64_t blk = c / DEC_SCAN;
      int64_t j[3] = {btop[3 * blk] + base_in[3 * c], btop[3 * blk + 1] + base_in[3 * c + 1], btop[3 * blk + 2] + base_in[3 * c + 2]};
      const int64_t r0 = r0_s;
      (void)dec_walk(d, ch, en, [&](int pos, int k) {
        const uint8_t* p = ch.b + pos + 4;   // the tag
        if (k == 0) {
          const int64_t r = j[0]++;
          const int64_t rl = r - r0;
          if (rl >= 0 && rl < maxrec) rpos[rl] = (uint16_t)(p - buf);
          ++nr;
          return;
        }
        const int64_t m = j[k]++;
        if (m >= o.marker_cap) { atomicExch(err, 2); return; }
        if (k == 1) {
          o.wm[m] = (int64_t)lds_be_u64(p + 1);
          o.wm_pos[m] = j[0];   // the records before it
        } else {   // latency marker: markedTime, then vertexId << 32 | subtaskIndex
          o.lm[2 * m] = (int64_t)lds_be_u64(p + 1);
          o.lm[2 * m + 1] = (int64_t)(((uint64_t)lds_be_u32(p + 9) << 32) | lds_be_u32(p + 13));
          o.lm_pos[m] = j[0];
        }
      });
    }
    if (nr) atomicAdd(&nrec_s, nr);
    __syncthreads();
    // the workgroup's records, in rank order
    const int nrec = min(nrec_s, maxrec);
    const int64_t r0 = r0_s;
    for (int rl = threadIdx.x; rl < nrec; rl += DEC_TW) {
      const int64_t r = r0 + rl;
      if (r >= o.record_cap) { atomicExch(err, 2); continue; }
      const uint8_t* p = buf + rpos[rl];
      const bool has_ts = p[0] == 0;
      const int64_t ts = has_ts ? (int64_t)lds_be_u64(p + 1) : INT64_MIN;
      const uint8_t* t = p + (has_ts ? 9 : 1);
      const int64_t key = d.key_int ? (int64_t)(int32_t)lds_be_u32(t + d.key_off) : (int64_t)lds_be_u64(t + d.key_off);
      o.key[r] = key;
      if (o.key_hash) o.key_hash[r] = (int32_t)key;   // Integer.hashCode
      o.ts[r] = ts;
      o.f1[r] = d.f1_off < 0 ? ts : d.f1_int ? (int64_t)(int32_t)lds_be_u32(t + d.f1_off) : (int64_t)lds_be_u64(t + d.f1_off);
      o.val[r] = (int64_t)lds_be_u64(t + d.val_off);
    }
  }
  // the last workgroup to finish posts the totals and the error word to the host (pinned, mapped): no copy after
  __syncthreads();
  if (threadIdx.x == 0 && atomicAdd(done, 1u) == gridDim.x - 1) {
    *done = 0u;
    for (int k = 0; k < 4; ++k) host_counts[k] = totals[k];
    host_counts[4] = (int64_t)atomicAdd(err, 0);
  }
}

}  // namespace fw

// enqueue one decode on the engine stream into scratch slot `slot`; its counts land in the slot's pinned words
// (event `done`).  *empty: nothing was enqueued (no bytes)
static int decode_enqueue(fw_engine* e, int slot, const fw_tuple_schema* sc, const void* bytes, int64_t nbytes,
                          int32_t mem, int64_t* key, int32_t* key_hash, int64_t* f1, int64_t* ts, void* value,
                          int64_t record_cap, int64_t* wm, int64_t* wm_pos, int64_t* lm, int64_t* lm_pos,
                          int64_t marker_cap, bool* empty) {
  using namespace fw;
  *empty = true;
  if (!e || !sc || (nbytes > 0 && !bytes) || nbytes < 0) return FW_ERR_INVALID_ARG;
  if (e->sticky) return e->sticky;
  fw_engine::DecSlot& ds = e->dec[slot];
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
  if (!ds.pin) {
    if (hipHostMalloc((void**)&ds.pin, 64, hipHostMallocMapped) != hipSuccess) {
      ds.pin = nullptr;
      return reject(e, FW_ERR_DEVICE, "decode: pinned count words");
    }
    HIPCHK(e, hipHostGetDevicePointer((void**)&ds.pin_dev, ds.pin, 0));
    HIPCHK(e, hipEventCreateWithFlags(&ds.done, hipEventDisableTiming));
  }
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
  const size_t nblk = (nc + DEC_SCAN - 1) / DEC_SCAN;
  const void* small_was = ds.small;
  HIPCHK(e, grow(ds.small, ds.small_cap, nc * (4 * DEC_W + 4 + 24 + 4 + 4 * DEC_W + 8 * DEC_S) + nblk * 24 + 256));
  const bool fresh = ds.small != small_was;   // (the workgroup arrival counter starts at zero)
  const uint8_t* src = (const uint8_t*)bytes;
  if (mem == FW_MEM_HOST) {
    HIPCHK(e, grow(ds.bytes, ds.bytes_cap, (size_t)nbytes));
    HIPCHK(e, hipMemcpyAsync(ds.bytes, bytes, (size_t)nbytes, hipMemcpyHostToDevice, e->stream));
    src = (const uint8_t*)ds.bytes;
  }
  d.bytes = src;
  uint8_t* sm = (uint8_t*)ds.small;
  unsigned int* done = (unsigned int*)sm;   // k_dec_emit's workgroup arrival counter (returns to 0): a fixed place
  int32_t* conv = (int32_t*)(sm + 16);      // [nc][DEC_W] each wave's agreeing exit
  int32_t* entry = conv + nc * DEC_W;
  int64_t* base = (int64_t*)(((uintptr_t)(entry + nc) + 7) & ~(uintptr_t)7);
  int64_t* totals = base + 3 * nc;   // [4] records, watermarks, latency markers, consumed bytes; then err
  int32_t* err = (int32_t*)(totals + 4);
  int64_t* btot = totals + 6;   // [3 nblk] block totals, then their exclusive offsets
  int32_t* cexit = (int32_t*)(btot + 3 * nblk);   // [nc] where each chunk's true chain leaves it
  int32_t* nsurv = cexit + nc;                     // [nc][DEC_W] survivors each wave found
  int64_t* surv = (int64_t*)(((uintptr_t)(nsurv + nc * DEC_W) + 7) & ~(uintptr_t)7);   // [nc][DEC_S] kept survivors
  if (fresh) HIPCHK(e, hipMemsetAsync(done, 0, 8, e->stream));
  const unsigned gb = (unsigned)((nc + DEC_T - 1) / DEC_T);
  // one workgroup per group (a persistent scan with the next group prefetched measured slower: 54 vs 47 us)
  hipLaunchKernelGGL(k_dec_scan, dim3(gb), dim3(DEC_TW), 0, e->stream, d, conv, surv, nsurv, err, (int64_t)gb);
  hipLaunchKernelGGL(k_dec_bscan, dim3((unsigned)nblk), dim3(DEC_SCAN), 0, e->stream, d, conv, surv, nsurv, entry, cexit,
                     base, btot, err);
  hipLaunchKernelGGL(k_dec_top, dim3(1), dim3(DEC_SCAN), 0, e->stream, d, entry, cexit, btot, (int64_t)nblk, totals);
  DecOut o{key, f1, ts, (int64_t*)value, wm, wm_pos, lm, lm_pos, key_hash, record_cap, marker_cap};
  // persistent: four workgroups per CU (dynamic LDS sized to the schema), at most one per group
  const unsigned eg = (unsigned)std::min<int64_t>((int64_t)gb, (int64_t)e->grid / 2);   // (grid = 8 per CU)
  hipLaunchKernelGGL(k_dec_emit, dim3(eg), dim3(DEC_TW), (size_t)2 * dec_maxrec(d.rec_len), e->stream, d, entry, base,
                     btot, o, err, totals, done, ds.pin_dev, (int64_t)gb);
  HIPCHK(e, hipGetLastError());
  HIPCHK(e, hipEventRecord(ds.done, e->stream));
  ds.record_cap = record_cap;
  ds.marker_cap = marker_cap;
  *empty = false;
  return FW_OK;
}

// wait for slot `slot`'s decode and report its counts
static int decode_finish(fw_engine* e, int slot, fw_decode_counts* out) {
  fw_engine::DecSlot& ds = e->dec[slot];
  HIPCHK(e, hipSetDevice(e->dev));
  HIPCHK(e, hipEventSynchronize(ds.done));
  const int64_t* tot = ds.pin;
  const int32_t herr = (int32_t)(tot[4] & 0xffffffff);
  if (herr == 1) return reject(e, FW_ERR_INVALID_ARG, "corrupt stream: no element chain through the bytes");
  out->n_records = tot[0];
  out->n_watermarks = tot[1];
  out->n_latency_markers = tot[2];
  out->consumed = tot[3];
  if (herr == 2 || tot[0] > ds.record_cap || tot[1] > ds.marker_cap || tot[2] > ds.marker_cap)
    return reject(e, FW_ERR_CAPACITY, "decode output capacity exceeded");
  return FW_OK;
}

int fw_decode(fw_engine* e, const fw_tuple_schema* sc, const void* bytes, int64_t nbytes, int32_t mem, int64_t* key,
              int32_t* key_hash, int64_t* f1, int64_t* ts, void* value, int64_t record_cap, int64_t* wm,
              int64_t* wm_pos, int64_t* lm, int64_t* lm_pos, int64_t marker_cap, fw_decode_counts* out) {
  if (!e || !out) return FW_ERR_INVALID_ARG;
  std::memset(out, 0, sizeof(*out));
  int slot = -1;
  for (int i = 0; i < fw_engine::NDEC && slot < 0; ++i) if (!e->dec[i].pending) slot = i;
  if (slot < 0) { e->err = "fw_decode: every decode slot has a decode outstanding (fw_decode_end first)"; return FW_ERR_INVALID_ARG; }
  bool empty = true;
  int rc = decode_enqueue(e, slot, sc, bytes, nbytes, mem, key, key_hash, f1, ts, value, record_cap, wm, wm_pos, lm, lm_pos,
                          marker_cap, &empty);
  if (rc || empty) return rc;
  return decode_finish(e, slot, out);
}

int fw_decode_begin(fw_engine* e, const fw_tuple_schema* sc, const void* bytes, int64_t nbytes, int32_t mem, int64_t* key,
                    int32_t* key_hash, int64_t* f1, int64_t* ts, void* value, int64_t record_cap, int64_t* wm,
                    int64_t* wm_pos, int64_t* lm, int64_t* lm_pos, int64_t marker_cap, int32_t* ticket) {
  if (!e || !ticket) return FW_ERR_INVALID_ARG;
  int slot = -1;   // the first free slot (decodes may end in any order)
  for (int i = 0; i < fw_engine::NDEC && slot < 0; ++i) if (!e->dec[i].pending) slot = i;
  if (slot < 0) { e->err = "fw_decode_begin: two decodes outstanding (fw_decode_end one first)"; return FW_ERR_INVALID_ARG; }
  fw_engine::DecSlot& ds = e->dec[slot];
  bool empty = true;
  int rc = decode_enqueue(e, slot, sc, bytes, nbytes, mem, key, key_hash, f1, ts, value, record_cap, wm, wm_pos, lm, lm_pos,
                          marker_cap, &empty);
  if (rc) return rc;
  ds.pending = true;
  ds.empty = empty;
  ds.ticket = (int32_t)(e->dec_seq++ & 0x7FFFFFFF);
  *ticket = ds.ticket;
  return FW_OK;
}

int fw_decode_end(fw_engine* e, int32_t ticket, fw_decode_counts* out) {
  if (!e || !out || ticket < 0) return FW_ERR_INVALID_ARG;
  std::memset(out, 0, sizeof(*out));
  int slot = -1;
  for (int i = 0; i < fw_engine::NDEC; ++i) if (e->dec[i].pending && e->dec[i].ticket == ticket) slot = i;
  if (slot < 0) { e->err = "fw_decode_end: no such decode outstanding"; return FW_ERR_INVALID_ARG; }
  e->dec[slot].pending = false;
  if (e->dec[slot].empty) return FW_OK;
  return decode_finish(e, slot, out);
}
