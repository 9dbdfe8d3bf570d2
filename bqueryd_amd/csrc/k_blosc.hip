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
// lists; here one wavefront decodes one split -- the stream's tokens are parsed by the whole
// wave in lock step from an LDS window of the compressed bytes, and every literal run and
// match is copied by the 64 lanes together -- and a second kernel un-shuffles the blocks.
#include <hip/hip_runtime.h>

#include <algorithm>

#include "blosc_gpu.h"

namespace bqg {

namespace {

constexpr int kWin = 1024;       // bytes of compressed input per wave in LDS
constexpr int kDecWaves = 4;     // waves per workgroup

__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// a 16-byte-aligned kWin-byte window of the compressed bytes in the wave's LDS, reloaded when
// the parse leaves it; every call is wave-uniform
struct Window {
  const unsigned char* src;  // the split's first compressed byte
  const unsigned char* base; // first byte of the window (16-byte aligned)
  unsigned char* win;
  int lane;
  __device__ __forceinline__ void load(uint32_t at) {
    base = reinterpret_cast<const unsigned char*>(reinterpret_cast<uintptr_t>(src + at) & ~(uintptr_t)15);
    // 16 bytes per lane; the staging buffer is padded by kBloscPad, so the window never
    // leaves the allocation
    const uint4 v = *reinterpret_cast<const uint4*>(base + lane * 16);
    *reinterpret_cast<uint4*>(win + lane * 16) = v;
    wave_lds_sync();
  }
  __device__ __forceinline__ uint32_t byte(uint32_t ip) {
    const unsigned char* p = src + ip;
    if (p < base || p >= base + kWin) load(ip);
    return win[p - base];
  }
};

__device__ __forceinline__ void copy_literals(const unsigned char* src, unsigned char* dst, uint32_t n, int lane) {
  for (uint32_t i = (uint32_t)lane; i < n; i += 64) dst[i] = src[i];
}

// a byte of this split's output, written earlier by this wave: an agent-scope load misses
// the (non-coherent) L1, which may hold a line fetched before the byte was stored
__device__ __forceinline__ unsigned char out_byte(const unsigned char* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// dst[i] = dst[i - dist] for i in [0, n): every byte comes from [dst - dist, dst), written
// before this match -- the wave's stores are drained (vmcnt counts stores on gfx9) first
__device__ __forceinline__ void copy_match(unsigned char* dst, uint32_t dist, uint32_t n, int lane) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  const unsigned char* ref = dst - dist;
  if (dist >= n) {
    for (uint32_t i = (uint32_t)lane; i < n; i += 64) dst[i] = out_byte(ref + i);
    return;
  }
  const uint32_t step = 64u % dist;
  uint32_t j = (uint32_t)lane % dist;
  for (uint32_t i = (uint32_t)lane; i < n; i += 64) {
    dst[i] = out_byte(ref + j);
    j += step;
    if (j >= dist) j -= dist;
  }
}

// LZ4 block format: [token][literal length ext][literals][offset u16 LE][match length ext]
__device__ uint32_t lz4_wave(Window& w, const unsigned char* src, uint32_t clen, unsigned char* dst, uint32_t dlen,
                             int lane) {
  uint32_t ip = 0, op = 0;
  while (ip < clen) {
    const uint32_t token = w.byte(ip++);
    uint32_t lit = token >> 4;
    if (lit == 15) {
      uint32_t b;
      do {
        if (ip >= clen) return 0xFFFFFFFFu;
        b = w.byte(ip++);
        lit += b;
      } while (b == 255);
    }
    if (ip + lit > clen || op + lit > dlen) return 0xFFFFFFFFu;
    copy_literals(src + ip, dst + op, lit, lane);
    ip += lit;
    op += lit;
    if (ip >= clen) break;  // the last sequence carries literals only
    if (ip + 2 > clen) return 0xFFFFFFFFu;
    const uint32_t off = w.byte(ip) | (w.byte(ip + 1) << 8);
    ip += 2;
    uint32_t mlen = token & 15u;
    if (mlen == 15) {
      uint32_t b;
      do {
        if (ip >= clen) return 0xFFFFFFFFu;
        b = w.byte(ip++);
        mlen += b;
      } while (b == 255);
    }
    mlen += 4;
    if (off == 0 || off > op || op + mlen > dlen) return 0xFFFFFFFFu;
    copy_match(dst + op, off, mlen, lane);
    op += mlen;
  }
  return op;
}

// BloscLZ (FastLZ-derived): ctrl < 32 -> ctrl + 1 literals; else a match of length
// (ctrl >> 5) + 2 (7: extended by bytes until one is not 255) at distance ((ctrl & 31) << 8)
// + next byte + 1, or 8192 + a big-endian u16 when that byte is 255 and ctrl & 31 == 31
constexpr uint32_t kBloscLzMaxDistance = 8191;

__device__ uint32_t blosclz_wave(Window& w, const unsigned char* src, uint32_t clen, unsigned char* dst,
                                 uint32_t dlen, int lane) {
  if (clen == 0) return 0;
  uint32_t ip = 0, op = 0;
  uint32_t ctrl = w.byte(ip++) & 31u;
  for (;;) {
    if (ctrl >= 32) {
      uint32_t len = (ctrl >> 5) - 1;
      uint32_t ofs = (ctrl & 31u) << 8;
      if (len == 6) {
        uint32_t code;
        do {
          if (ip + 1 >= clen) return 0xFFFFFFFFu;
          code = w.byte(ip++);
          len += code;
        } while (code == 255);
      } else if (ip + 1 >= clen) {
        return 0xFFFFFFFFu;
      }
      const uint32_t code = w.byte(ip++);
      len += 3;
      uint32_t dist = ofs + code + 1;
      if (code == 255 && ofs == (31u << 8)) {
        if (ip + 1 >= clen) return 0xFFFFFFFFu;
        ofs = (w.byte(ip) << 8) + w.byte(ip + 1);
        ip += 2;
        dist = ofs + kBloscLzMaxDistance + 1;
      }
      if (op + len > dlen || dist > op) return 0xFFFFFFFFu;
      copy_match(dst + op, dist, len, lane);
      op += len;
      if (ip >= clen) break;
      ctrl = w.byte(ip++);
    } else {
      const uint32_t n = ctrl + 1;
      if (op + n > dlen || ip + n > clen) return 0xFFFFFFFFu;
      copy_literals(src + ip, dst + op, n, lane);
      op += n;
      ip += n;
      if (ip >= clen) break;
      ctrl = w.byte(ip++);
    }
  }
  return op;
}

}  // namespace

__global__ __launch_bounds__(64 * kDecWaves) void k_blosc_decode(const unsigned char* comp, const BloscSplit* tasks,
                                                                 int ntasks, unsigned int* bad) {
  __shared__ __align__(16) unsigned char win_all[kDecWaves][kWin];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  Window w;
  w.base = nullptr;
  w.win = win_all[wave];
  w.lane = lane;
  for (int t = blockIdx.x * kDecWaves + wave; t < ntasks; t += gridDim.x * kDecWaves) {
    const BloscSplit s = tasks[t];
    const unsigned char* src = comp + s.src;
    unsigned char* dst = reinterpret_cast<unsigned char*>(s.dst);
    uint32_t got;
    if (s.codec == kSplitRaw) {
      copy_literals(src, dst, s.dsize, lane);
      got = s.dsize;
    } else {
      w.src = src;
      w.load(0);
      got = s.codec == kSplitLz4 ? lz4_wave(w, src, s.csize, dst, s.dsize, lane)
                                 : blosclz_wave(w, src, s.csize, dst, s.dsize, lane);
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
  const int blocks = std::min(65535, (ntasks + kDecWaves - 1) / kDecWaves);
  hipLaunchKernelGGL(k_blosc_decode, dim3(blocks), dim3(64 * kDecWaves), 0, st, comp, tasks, ntasks, bad);
}

void launch_blosc_unshuffle(const BloscBlock* blocks, int nblocks, hipStream_t st) {
  if (nblocks <= 0) return;
  hipLaunchKernelGGL(k_blosc_unshuffle, dim3(std::min(nblocks, 65535)), dim3(256), 0, st, blocks, nblocks);
}

}  // namespace bqg
