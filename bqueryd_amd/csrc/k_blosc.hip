// k_blosc.hip -- on-GPU decode of bcolz chunks (blosc1 frames): the compressed bytes cross
// PCIe instead of the decoded ones, and host cores only read files.
//
// A blosc1 frame [ext-bcolz / c-blosc 1.x format, unverified: c-blosc is not vendored, only
// its shared library is present; checked against that library's own decode by the tests]:
//   16-byte header: version, versionlz, flags (bit 0 byte shuffle, bit 1 memcpyed, bit 2 bit
//   shuffle, bit 4 "blocks not split", bits 5-7 codec: 0 BloscLZ, 1 LZ4), typesize, nbytes,
//   blocksize, cbytes (little-endian int32); then, unless memcpyed, one int32 start offset
//   per block; a block holds `typesize` splits when it is a full block, typesize <= 16,
//   blocksize / typesize >= 128 and bit 4 is clear (else 1 split); each split is an int32
//   compressed size and the codec's stream (stored raw when the size equals the split's
//   decoded size); a byte-shuffled block is `typesize` planes of blocksize / typesize bytes.
// The host (ingest.hip) parses headers and split sizes into BloscSplit / BloscBlock task
// lists; here one wavefront decodes one split (LZ4 or BloscLZ) -- up to 64 sequences at a
// time, one per lane, found by a speculative parse and pointer doubling (see the LZ4 section);
// long runs and matches are copied by the 64 lanes together -- and a second kernel
// un-shuffles the blocks.
#include <hip/hip_runtime.h>

#include <algorithm>

#include "blosc_gpu.h"

namespace bqg {

namespace {

constexpr int kWin = 1024;        // bytes of compressed input per wave in LDS
constexpr uint32_t kRing = 32768; // bytes of decoded history per wave in LDS
// one wave per workgroup, 33 KiB of LDS each: 4 waves per CU

// address-space-qualified pointers: global (not flat) loads and stores, so an LDS wait
// (lgkmcnt) never waits for the wave's outstanding global stores as well
typedef __attribute__((address_space(1))) unsigned char gbyte;
typedef __attribute__((address_space(3))) unsigned char lbyte;
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ uint32_t uniform(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }

// The split's compressed bytes: a 16-byte-aligned kWin-byte window of them in the wave's LDS
// (reloaded when the parse leaves it) and a cursor `ip` that hands out header bytes from an
// 8-byte register copy, so a token costs one LDS round trip, not one per byte.  Every call
// is wave-uniform.
struct Window {
  const gbyte* src;  // the split's first compressed byte
  lbyte* win;
  int32_t lo;        // split offset of the window's first byte (may be < 0: alignment)
  int lane;
  uint32_t ip;       // cursor: offset of the next byte in the split
  uint64_t q;        // bytes [ip, ip + have) of the split, low byte first
  uint32_t have;

  __device__ __forceinline__ void load(uint32_t at) {
    const uint32_t mis = (uint32_t)(reinterpret_cast<uintptr_t>(src + at) & 15);
    lo = (int32_t)uniform(at - mis);
    // 16 bytes per lane; the staging buffer is padded by kBloscPad, so the window never
    // leaves the allocation
    const u32x4 v = *(const __attribute__((address_space(1))) u32x4*)(src + lo + lane * 16);
    *(__attribute__((address_space(3))) u32x4*)(win + lane * 16) = v;
    wave_lds_sync();
  }
  // the window covers split bytes [ip + at, ip + at + n); returns the first one's LDS offset
  __device__ __forceinline__ uint32_t cover(uint32_t at, uint32_t n) {
    const int32_t p = (int32_t)(ip + at);
    if (p < lo || p + (int32_t)n > lo + kWin) load(ip + at);
    return (uint32_t)(p - lo);
  }
  __device__ __forceinline__ void fill() {
    const uint32_t off = cover(0, 16);
    const __attribute__((address_space(3))) uint64_t* w64 = (const __attribute__((address_space(3))) uint64_t*)(win);
    const uint64_t a = w64[off >> 3], b = w64[(off >> 3) + 1];
    const uint32_t sh = (off & 7) * 8;
    const uint64_t v = sh ? (a >> sh) | (b << (64 - sh)) : a;
    q = ((uint64_t)uniform((uint32_t)(v >> 32)) << 32) | uniform((uint32_t)v);
    have = 8;
  }
  __device__ __forceinline__ uint32_t next() {
    if (!have) fill();
    const uint32_t b = (uint32_t)q & 255u;
    q >>= 8;
    --have;
    ++ip;
    return b;
  }
  __device__ __forceinline__ void skip(uint32_t n) {
    if (n < have) {
      q >>= 8 * n;
      have -= n;
    } else {
      have = 0;
    }
    ip += n;
  }
};

// The wave's output: global bytes plus the last kRing of them in LDS.  A match whose source
// lies in that history is copied LDS -> registers -> global without waiting for the wave's
// global stores; only a match reaching further back waits for them (vmcnt) and reads the
// output through L2.
struct Out {
  gbyte* dst;   // the split's output (global)
  lbyte* ring;  // kRing bytes of LDS: position p lives at ring[p % kRing]
  int lane;
  __device__ __forceinline__ void put(uint32_t p, unsigned char v) {
    dst[p] = v;
    ring[p & (kRing - 1)] = v;
  }
};

// n literal bytes at the cursor -> output position op
__device__ __forceinline__ void copy_literals(Window& w, Out& o, uint32_t op, uint32_t n) {
  for (uint32_t c = 0; c < n; c += 64) {
    const uint32_t off = w.cover(c, 64);
    const uint32_t i = c + (uint32_t)o.lane;
    if (i < n) o.put(op + i, w.win[off + o.lane]);
  }
  wave_lds_sync();
  w.skip(n);
}

// a byte of this split's output, written earlier by this wave: an agent-scope load misses
// the (non-coherent) L1, which may hold a line fetched before the byte was stored
__device__ __forceinline__ unsigned char out_byte(const gbyte* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// out[op + i] = out[op + i - dist] for i in [0, n)
__device__ __forceinline__ void copy_match(Out& o, uint32_t op, uint32_t dist, uint32_t n) {
  const uint32_t lane = (uint32_t)o.lane;
  if (dist == 1 && n >= 2048) {
    // a long run of one byte (the zero planes of shuffled integers): 16-byte stores, and only
    // the last kRing bytes go to the history
    const uint32_t v = o.ring[(op - 1) & (kRing - 1)];
    const uint32_t v4 = v * 0x01010101u;
    gbyte* d = o.dst + op;
    const uint32_t head = (uint32_t)((16 - (reinterpret_cast<uintptr_t>(d) & 15)) & 15);
    if (lane < head) d[lane] = (unsigned char)v;
    const uint32_t body = (n - head) & ~15u;
    typedef __attribute__((address_space(1))) u32x4 g32x4;
    g32x4* d16 = (g32x4*)(d + head);
    const u32x4 w = {v4, v4, v4, v4};
    for (uint32_t i = lane; i < body / 16; i += 64) d16[i] = w;
    for (uint32_t i = head + body + lane; i < n; i += 64) d[i] = (unsigned char)v;
    if (n >= kRing) {  // the whole history becomes this byte
      typedef __attribute__((address_space(3))) u32x4 l32x4;
      l32x4* r16 = (l32x4*)o.ring;
      for (uint32_t i = lane; i < kRing / 16; i += 64) r16[i] = w;
    } else {
      for (uint32_t i = lane; i < n; i += 64) o.ring[(op + i) & (kRing - 1)] = (unsigned char)v;
    }
    wave_lds_sync();
    return;
  }
  if (dist <= 64) {
    // the period [op - dist, op) in registers, then byte i = period[i mod dist] by lane
    // permute: no reads of bytes written by this match
    const uint32_t per = o.ring[(op - dist + lane % dist) & (kRing - 1)];
    const uint32_t step = 64u % dist;
    uint32_t j = lane % dist;
    for (uint32_t c = 0; c < n; c += 64) {
      const uint32_t v = (uint32_t)__shfl((int)per, (int)j, 64);
      if (c + lane < n) o.put(op + c + lane, (unsigned char)v);
      j += step;
      if (j >= dist) j -= dist;
    }
  } else if (dist <= kRing) {
    // sources at least 64 back: a 64-byte step reads only bytes of earlier steps, still in
    // the ring (a byte is overwritten kRing positions later)
    for (uint32_t c = 0; c < n; c += 64) {
      const uint32_t i = c + lane;
      if (i < n) o.put(op + i, o.ring[(op + i - dist) & (kRing - 1)]);
      if (c + 128 > dist) wave_lds_sync();  // the next step reads this one's bytes
    }
  } else {
    // far back: through global memory once the wave's stores have drained
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    for (uint32_t c = 0; c < n; c += 64) {
      const uint32_t i = c + lane;
      if (i < n) o.put(op + i, out_byte(o.dst + op + i - dist));
      if (c + 128 > dist) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // sources of the next step
    }
  }
  wave_lds_sync();
}

constexpr uint32_t kBad = 0xFFFFFFFFu;

#ifdef BQG_BLOSC_PROF
// micro-benchmark instrumentation (tools/micro): cycles and counts per phase of the LZ4 loop
__device__ unsigned long long g_blosc_prof[32];
#define PROF_DECL uint64_t prof_t = __builtin_readcyclecounter(), prof_acc[8] = {}, prof_n[8] = {}
#define PROF_MARK(k)                                      \
  do {                                                    \
    const uint64_t now_ = __builtin_readcyclecounter();   \
    prof_acc[k] += now_ - prof_t;                         \
    prof_n[k] += 1;                                       \
    prof_t = now_;                                        \
  } while (0)
#define PROF_FLUSH                                                                   \
  do {                                                                               \
    if (o.lane == 0)                                                                 \
      for (int k_ = 0; k_ < 8; ++k_) {                                               \
        atomicAdd(&g_blosc_prof[k_], (unsigned long long)prof_acc[k_]);              \
        atomicAdd(&g_blosc_prof[16 + k_], (unsigned long long)prof_n[k_]);           \
      }                                                                              \
  } while (0)
#else
#define PROF_DECL
#define PROF_MARK(k)
#define PROF_FLUSH
#endif

// ---- LZ4 ------------------------------------------------------------------------------
// Block format: sequences [token][literal length ext][literals][offset u16 LE][match length
// ext]; the last sequence carries literals only.
//
// A sequence costs the serial loop one or two LDS round trips (its header, its match source),
// which leaves a wave at ~1000 cycles per sequence on low-entropy planes (~22 K sequences per
// 128 KiB split).  So sequences are decoded in groups of up to 64, one per lane:
//  1. every lane parses the sequence that would start at each of 4 candidate offsets of the
//     next kSpan compressed bytes (speculative: most candidates are not sequence starts);
//  2. the true chain of starts through those parses is found by pointer doubling over the
//     candidates' next-start table (lane permutes), up to 64 sequences / kGroupOut bytes;
//  3. each sequence's lane writes its literals into the LDS history, then the matches run in
//     rounds -- a match whose source lies wholly before the first unfinished match's start
//     is final and copies (lane-serially, 4 bytes per LDS round trip);
//  4. the group's decoded bytes are stored from the history to global memory, coalesced.
// Long literal runs / matches (> kLong) and sequences not wholly inside the window go through
// the wave-cooperative serial path, one at a time.
constexpr uint32_t kSpan = 256;
constexpr uint32_t kGroupOut = 4096;
constexpr uint32_t kLong = 64;
constexpr uint32_t kRingSafe = kRing - kGroupOut;  // group matches reaching further read global
constexpr uint32_t kNone = 0xFFFFFFFFu;
constexpr uint32_t kDead = 1024;  // jump-table mark of a non-sequence candidate (> any next)

// one sequence at the cursor, wave-cooperative; returns the new output position or kBad
__device__ uint32_t lz4_one(Window& w, uint32_t clen, Out& o, uint32_t op, uint32_t dlen) {
  const uint32_t token = w.next();
  uint32_t lit = token >> 4;
  if (lit == 15) {
    uint32_t b;
    do {
      if (w.ip >= clen) return kBad;
      b = w.next();
      lit += b;
    } while (b == 255);
  }
  if (w.ip + lit > clen || op + lit > dlen) return kBad;
  if (lit) copy_literals(w, o, op, lit);
  op += lit;
  if (w.ip >= clen) return op;  // the last sequence
  if (w.ip + 2 > clen) return kBad;
  const uint32_t lo = w.next();
  const uint32_t off = lo | (w.next() << 8);
  uint32_t mlen = token & 15u;
  if (mlen == 15) {
    uint32_t b;
    do {
      if (w.ip >= clen) return kBad;
      b = w.next();
      mlen += b;
    } while (b == 255);
  }
  mlen += 4;
  if (off == 0 || off > op || op + mlen > dlen) return kBad;
  copy_match(o, op, off, mlen);
  return op + mlen;
}

struct Seq {
  uint32_t next;    // split offset after the sequence; kNone: not a group sequence (not wholly
                    // inside window and split, or a literal run / match longer than kLong)
  uint32_t lit;     // literal bytes
  uint32_t litpos;  // split offset of the literals
  uint32_t dist;    // match offset (0: the last sequence)
  uint32_t mlen;    // match bytes
};

// bytes [rel, rel + 4) of the window, little-endian: two aligned dword reads (the window
// array is padded by 16 bytes)
__device__ __forceinline__ uint32_t peek4(const lbyte* win, uint32_t rel) {
  const __attribute__((address_space(3))) uint32_t* w32 = (const __attribute__((address_space(3))) uint32_t*)(win);
  const uint32_t a = w32[rel >> 2], b = w32[(rel >> 2) + 1];
  return __builtin_amdgcn_alignbyte(b, a, rel & 3);
}

// the sequence that would start at split offset c, parsed from the window (per lane): two
// dependent LDS round trips -- the header word, then the offset word past the literals
__device__ __forceinline__ Seq lz4_seq_at(const Window& w, uint32_t c, uint32_t clen) {
  Seq s = {kNone, 0, 0, 0, 0};
  const int32_t rel = (int32_t)c - w.lo;
  if (c >= clen || rel < 0 || rel >= kWin) return s;
  const uint32_t end = min(clen - c, (uint32_t)(kWin - rel));  // bytes readable from c
  const uint32_t h = peek4(w.win, (uint32_t)rel);
  const uint32_t token = h & 255u;
  uint32_t q = 1, lit = token >> 4;
  if (lit == 15) {  // one extension byte at most: longer runs are not group sequences
    if (end < 2) return s;
    const uint32_t x = (h >> 8) & 255u;
    lit += x;
    q = 2;
    if (x == 255) return s;
  }
  if (lit > kLong || lit > end - q) return s;
  s.litpos = c + q;
  s.lit = lit;
  q += lit;
  if (q == clen - c) {  // the last sequence
    s.next = clen;
    return s;
  }
  if (q + 2 > end) return s;
  const uint32_t g = peek4(w.win, (uint32_t)rel + q);
  s.dist = g & 0xFFFFu;
  q += 2;
  uint32_t m = token & 15u;
  if (m == 15) {
    if (q >= end) return s;
    const uint32_t x = (g >> 16) & 255u;
    m += x;
    ++q;
    if (x == 255) return s;
  }
  s.mlen = m + 4;
  if (s.mlen > kLong) return s;
  s.next = c + q;
  return s;
}

// inclusive prefix sum over the wave: DPP row shifts, then row broadcasts
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t x) {
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xF, 0xF, false);  // row_shr:1
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xF, 0xF, false);  // row_shr:2
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xF, 0xF, false);  // row_shr:4
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xF, 0xF, false);  // row_shr:8
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xA, 0xF, false);  // row_bcast:15
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xC, 0xF, false);  // row_bcast:31
  return x;
}

// ---- BloscLZ ---------------------------------------------------------------------------
// FastLZ-derived tokens: ctrl < 32 -> ctrl + 1 literals; else a match of length (ctrl >> 5) + 2
// (7: extended by bytes until one is not 255) at distance ((ctrl & 31) << 8) + next byte + 1,
// or 8192 + a big-endian u16 when that byte is 255 and ctrl & 31 == 31.  The first token is a
// literal run of (first byte & 31) + 1.  A match needs at least one byte after its distance
// byte (the stream ends with literals).  The group decoder below treats a token as a sequence
// with either literals or a match.
constexpr uint32_t kBloscLzMaxDistance = 8191;

// one token at the cursor (not the first), wave-cooperative; the new output position or kBad
__device__ uint32_t blosclz_one(Window& w, uint32_t clen, Out& o, uint32_t op, uint32_t dlen) {
  const uint32_t ctrl = w.next();
  if (ctrl < 32) {
    const uint32_t n = ctrl + 1;
    if (op + n > dlen || w.ip + n > clen) return kBad;
    copy_literals(w, o, op, n);
    return op + n;
  }
  uint32_t len = (ctrl >> 5) - 1;
  uint32_t ofs = (ctrl & 31u) << 8;
  if (len == 6) {
    uint32_t code;
    do {
      if (w.ip + 1 >= clen) return kBad;
      code = w.next();
      len += code;
    } while (code == 255);
  } else if (w.ip + 1 >= clen) {
    return kBad;
  }
  const uint32_t code = w.next();
  len += 3;
  uint32_t dist = ofs + code + 1;
  if (code == 255 && ofs == (31u << 8)) {
    if (w.ip + 1 >= clen) return kBad;
    const uint32_t hi = w.next();
    ofs = (hi << 8) + w.next();
    dist = ofs + kBloscLzMaxDistance + 1;
  }
  if (op + len > dlen || dist > op) return kBad;
  copy_match(o, op, dist, len);
  return op + len;
}

// the token that would start at split offset c (not the first), parsed from the window
__device__ __forceinline__ Seq blosclz_seq_at(const Window& w, uint32_t c, uint32_t clen) {
  Seq s = {kNone, 0, 0, 0, 0};
  const int32_t rel = (int32_t)c - w.lo;
  if (c >= clen || rel < 0 || rel >= kWin) return s;
  const uint32_t avail = clen - c;                 // bytes to the end of the stream
  const uint32_t wend = (uint32_t)(kWin - rel);    // bytes to the end of the window
  const uint64_t hb = (uint64_t)peek4(w.win, (uint32_t)rel) | ((uint64_t)peek4(w.win, (uint32_t)rel + 4) << 32);
  const uint32_t ctrl = (uint32_t)hb & 255u;
  if (ctrl < 32) {
    const uint32_t n = ctrl + 1;
    if (1 + n > min(avail, wend)) return s;
    s.lit = n;
    s.litpos = c + 1;
    s.next = c + 1 + n;
    return s;
  }
  uint32_t len = (ctrl >> 5) - 1, ofs = (ctrl & 31u) << 8, q = 1;
  if (len == 6) {  // one extension byte at most: longer matches are not group sequences
    if (q + 1 >= avail) return s;
    const uint32_t x = (uint32_t)(hb >> (8 * q)) & 255u;
    ++q;
    len += x;
    if (x == 255) return s;
  } else if (q + 1 >= avail) {
    return s;
  }
  const uint32_t code = (uint32_t)(hb >> (8 * q)) & 255u;
  ++q;
  uint32_t dist = ofs + code + 1;
  if (code == 255 && ofs == (31u << 8)) {
    if (q + 1 >= avail) return s;
    dist = ((((uint32_t)(hb >> (8 * q)) & 255u) << 8) | ((uint32_t)(hb >> (8 * q + 8)) & 255u)) + kBloscLzMaxDistance + 1;
    q += 2;
  }
  if (q > wend || len + 3 > kLong) return s;
  s.dist = dist;
  s.mlen = len + 3;
  s.next = c + q;
  return s;
}

// D(x) for a jump table held as 4 x 64 lanes (entry x at lane x % 64 of register x / 64):
// every lane gathers its own x by lane permute; x >= kSpan (left the span, or dead) is fixed
__device__ __forceinline__ uint32_t jump(const uint32_t (&tbl)[4], uint32_t x) {
  const int l = (int)(x & 63);
  const uint32_t a = (uint32_t)__shfl((int)tbl[0], l, 64), b = (uint32_t)__shfl((int)tbl[1], l, 64);
  const uint32_t c = (uint32_t)__shfl((int)tbl[2], l, 64), d = (uint32_t)__shfl((int)tbl[3], l, 64);
  const uint32_t k = x >> 6;
  const uint32_t v = k == 0 ? a : k == 1 ? b : k == 2 ? c : d;
  return x < kSpan ? v : x;
}

// LZ4 (BLZ false) or BloscLZ (BLZ true) stream, decoded in groups of sequences
template <bool BLZ>
__device__ uint32_t group_wave(Window& w, uint32_t clen, Out& o, uint32_t dlen) {
  const uint32_t lane = (uint32_t)o.lane;
  constexpr uint32_t M = kRing - 1;
  uint32_t op = 0;
  PROF_DECL;
  if (BLZ) {  // the first token: a literal run of (first byte & 31) + 1
    if (clen == 0) return 0;
    const uint32_t n = (w.next() & 31u) + 1;
    if (n > dlen || w.ip + n > clen) return kBad;
    copy_literals(w, o, 0, n);
    op = n;
  }
  while (w.ip < clen) {
    const uint32_t ip = w.ip;
    // 1. speculative parses of the candidate starts ip + 64 k + lane
    w.cover(0, kSpan + 2 * kLong);
    // jump table D0 over the 4 x 64 candidates: the next start relative to ip (>= kSpan: the
    // chain leaves the span), or kDead + c for a candidate that is not a group sequence
    uint32_t d[6][4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const uint32_t c = 64 * k + lane;
      const Seq s = BLZ ? blosclz_seq_at(w, ip + c, clen) : lz4_seq_at(w, ip + c, clen);
      d[0][k] = s.next == kNone ? kDead + c : s.next - ip;
    }
    PROF_MARK(0);
    // 2. the chain of true starts by pointer doubling: D(j+1) = D(j) o D(j), then lane i
    //    composes the D(j) of the bits of i: e_i = D0^i(0), the i-th sequence start
#pragma unroll
    for (int j = 1; j < 6; ++j)
#pragma unroll
      for (int k = 0; k < 4; ++k) d[j][k] = jump(d[j - 1], d[j - 1][k]);
    uint32_t e = 0;
#pragma unroll
    for (int j = 0; j < 6; ++j) {
      const uint32_t f = jump(d[j], e);
      if ((lane >> j) & 1) e = f;
    }
    const uint32_t en = jump(d[0], e);  // the start after e_i
    uint32_t t = (uint32_t)__builtin_popcountll(__ballot(e < kSpan && en < kDead));
    PROF_MARK(1);
    if (t == 0) {
      op = BLZ ? blosclz_one(w, clen, o, op, dlen) : lz4_one(w, clen, o, op, dlen);
      if (op == kBad) return kBad;
      PROF_MARK(7);
      continue;
    }
    // 3. the group: one sequence per lane (at most kGroupOut decoded bytes)
    Seq s = {0, 0, 0, 0, 0};
    if (lane < t) s = BLZ ? blosclz_seq_at(w, ip + e, clen) : lz4_seq_at(w, ip + e, clen);
    const uint32_t sz = s.lit + s.mlen;
    const uint32_t incl = wave_incl_scan(sz);
    t = max(1u, min(t, (uint32_t)__builtin_popcountll(__ballot(incl <= kGroupOut))));
    const bool act = lane < t;
    if (!act) s = Seq{0, 0, 0, 0, 0};
    const uint32_t out = __builtin_amdgcn_readlane(incl, t - 1);
    const uint32_t p = ip + __builtin_amdgcn_readlane(en, t - 1);
    const uint32_t ostart = op + incl - sz, ms = ostart + s.lit;
    const bool bad = act && (ms + s.mlen > dlen || (s.mlen && (s.dist == 0 || s.dist > ms)));
    if (__ballot(bad)) return kBad;
    PROF_MARK(2);
    if (act && s.lit) {
      const lbyte* lsrc = w.win + (s.litpos - w.lo);
      for (uint32_t j = 0; j < s.lit; ++j) o.ring[(ostart + j) & M] = lsrc[j];
    }
    if (__ballot(act && s.mlen && s.dist > kRingSafe)) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    wave_lds_sync();
    PROF_MARK(3);
    uint64_t pend = __ballot(act && s.mlen != 0);
    while (pend) {
      const uint32_t u = (uint32_t)__builtin_ctzll(pend);
      const uint32_t F = __builtin_amdgcn_readlane(ms, u);
      const bool ready = ((pend >> lane) & 1) && ms - s.dist + min(s.mlen, s.dist) <= F;
      if (ready) {
        const uint32_t src = ms - s.dist;
        if (s.dist > kRingSafe) {
          for (uint32_t j = 0; j < s.mlen; ++j) o.ring[(ms + j) & M] = out_byte(o.dst + src + j);
        } else if (s.dist >= 4) {
          for (uint32_t j = 0; j < s.mlen; j += 4) {
            const uint32_t b0 = o.ring[(src + j) & M], b1 = o.ring[(src + j + 1) & M];
            const uint32_t b2 = o.ring[(src + j + 2) & M], b3 = o.ring[(src + j + 3) & M];
            o.ring[(ms + j) & M] = (unsigned char)b0;
            if (j + 1 < s.mlen) o.ring[(ms + j + 1) & M] = (unsigned char)b1;
            if (j + 2 < s.mlen) o.ring[(ms + j + 2) & M] = (unsigned char)b2;
            if (j + 3 < s.mlen) o.ring[(ms + j + 3) & M] = (unsigned char)b3;
          }
        } else {
          for (uint32_t j = 0; j < s.mlen; ++j) o.ring[(ms + j) & M] = o.ring[(src + j) & M];
        }
      }
      wave_lds_sync();
      pend &= ~__ballot(ready);
      PROF_MARK(5);
    }
    PROF_MARK(4);
    // 4. the group's bytes to global memory
    for (uint32_t c = 0; c < out; c += 64)
      if (c + lane < out) o.dst[op + c + lane] = o.ring[(op + c + lane) & M];
    op += out;
    w.ip = p;
    w.have = 0;
    PROF_MARK(6);
  }
  PROF_FLUSH;
  return op;
}

}  // namespace

__global__ __launch_bounds__(64) void k_blosc_decode(const unsigned char* comp, const BloscSplit* tasks, int ntasks,
                                                     unsigned int* bad) {
  __shared__ __align__(16) unsigned char win_s[kWin + 16];
  __shared__ __align__(16) unsigned char ring_s[kRing];
  const int lane = threadIdx.x;
  Window w;
  w.win = (lbyte*)(win_s);
  w.lane = lane;
  Out o;
  o.ring = (lbyte*)(ring_s);
  o.lane = lane;
  const gbyte* gcomp = (const gbyte*)(comp);
  for (int t = blockIdx.x; t < ntasks; t += gridDim.x) {
    const BloscSplit s = tasks[t];
    const gbyte* src = gcomp + s.src;
    o.dst = (gbyte*)(s.dst);
    uint32_t got;
    if (s.codec == kSplitRaw) {
      for (uint32_t i = (uint32_t)lane; i < s.dsize; i += 64) o.dst[i] = src[i];
      got = s.dsize;
    } else {
      w.src = src;
      w.ip = 0;
      w.have = 0;
      w.load(0);
      got = s.codec == kSplitLz4 ? group_wave<false>(w, s.csize, o, s.dsize) : group_wave<true>(w, s.csize, o, s.dsize);
    }
    if (got != s.dsize && lane == 0) atomicOr(bad, 1u);  // a vector atomic (one lane)
  }
}

// byte un-shuffle: block bytes are `typesize` planes of n = size / typesize bytes (plane j
// holds byte j of every element); trailing size % typesize bytes are stored as they are.
// Element-sized stores for the common type sizes (block offsets are multiples of typesize).
template <typename T>
__device__ __forceinline__ void unshuffle_typed(const unsigned char* s, unsigned char* d, uint32_t n) {
  constexpr uint32_t ts = sizeof(T);
  for (uint32_t e = threadIdx.x; e < n; e += blockDim.x) {
    T v = 0;
#pragma unroll
    for (uint32_t j = 0; j < ts; ++j) v |= (T)s[(size_t)j * n + e] << (8 * j);
    reinterpret_cast<T*>(d)[e] = v;
  }
}

__global__ __launch_bounds__(256) void k_blosc_unshuffle(const BloscBlock* blocks, int nblocks) {
  for (int b = blockIdx.x; b < nblocks; b += gridDim.x) {
    const BloscBlock k = blocks[b];
    const unsigned char* s = reinterpret_cast<const unsigned char*>(k.tmp);
    unsigned char* d = reinterpret_cast<unsigned char*>(k.dst);
    const uint32_t ts = k.typesize, n = k.bytes / ts;
    if (ts == 2)
      unshuffle_typed<uint16_t>(s, d, n);
    else if (ts == 4)
      unshuffle_typed<uint32_t>(s, d, n);
    else if (ts == 8)
      unshuffle_typed<uint64_t>(s, d, n);
    else
      for (uint32_t e = threadIdx.x; e < n; e += blockDim.x)
        for (uint32_t j = 0; j < ts; ++j) d[(size_t)e * ts + j] = s[(size_t)j * n + e];
    for (uint32_t r = n * ts + threadIdx.x; r < k.bytes; r += blockDim.x) d[r] = s[r];
  }
}

void launch_blosc_decode(const unsigned char* comp, const BloscSplit* tasks, int ntasks, unsigned int* bad,
                         hipStream_t st) {
  if (ntasks <= 0) return;
  hipLaunchKernelGGL(k_blosc_decode, dim3(std::min(65535, ntasks)), dim3(64), 0, st, comp, tasks, ntasks, bad);
}

void launch_blosc_unshuffle(const BloscBlock* blocks, int nblocks, hipStream_t st) {
  if (nblocks <= 0) return;
  hipLaunchKernelGGL(k_blosc_unshuffle, dim3(std::min(nblocks, 65535)), dim3(256), 0, st, blocks, nblocks);
}

}  // namespace bqg
