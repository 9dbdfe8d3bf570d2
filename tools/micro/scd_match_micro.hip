// scd_match_micro.hip -- the C4 random-order step in isolation: how a wave finds the lanes of
// each slot in a 64-row step (sorted_count_distinct needs each row's previous row of the same
// slot, and one state update per slot).  Two variants over the same rows, checked against each
// other and a host reference (per-slot rows and value changes):
//   0  LDS lane masks (the library's k_scd_fused, scd.h): every lane ORs its bit into its slot's
//      64-bit mask word in wave-private LDS and reads it back; the slot's first lane updates the
//      slot state, its last lane stores the new last value;
//   1  wave-local counting sort: a stable LSD radix sort of the step's (slot, lane) pairs by
//      slot, one bit per pass (ballot + mbcnt ranks, ds_permute moves; no LDS bank traffic),
//      then every slot is a contiguous run of sorted lanes: the previous row of a slot is the
//      sorted lane below (a DPP shift), the run head updates the state, the run tail stores
//      the last value -- two random LDS accesses per slot instead of three per row.
// Rows: C4's shape (265 pickup locations, passenger_count values 0..9), random order; one wave
// per 64 Ki-row chunk, 20-byte-per-slot wave state as in the compact library kernel.
// build: hipcc -O3 -std=c++17 --offload-arch=gfx950 tools/micro/scd_match_micro.hip -o tools/micro/bin/scd_match_micro
// run:   scd_match_micro [rows] [reps]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                  \
    }                                                                           \
  } while (0)

constexpr int kSlots = 265;
constexpr int kSlotBits = 9;
constexpr int kWaves = 4;                // per 256-thread workgroup
constexpr uint32_t kChunk = 65280;       // rows per wave (16-bit row / change counters)

struct State {  // per slot and wave
  uint32_t last;
  uint32_t rc;  // rows | changes << 16
};

__device__ __forceinline__ uint32_t mbcnt64(uint64_t m) {
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

template <int VARIANT>
__global__ __launch_bounds__(256) void k_match(const uint16_t* slot, const uint8_t* val, uint32_t nrows,
                                               uint32_t* out_rows, uint32_t* out_changes) {
  __shared__ State st_all[kWaves][kSlots];
  __shared__ unsigned long long tbl_all[kWaves][kSlots];
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  State* st = st_all[wave];
  unsigned long long* tbl = tbl_all[wave];
  for (int i = lane; i < kSlots; i += 64) {
    st[i] = State{0u, 0u};
    tbl[i] = 0ull;
  }
  __builtin_amdgcn_s_waitcnt(0xc07f);
  const uint32_t w = blockIdx.x * kWaves + wave;
  const uint32_t start = w * kChunk;
  const uint32_t end = min(nrows, start + kChunk);
  const uint64_t lanes_below = (1ull << lane) - 1ull;
  for (uint32_t base = start; base < end; base += 64) {
    const uint32_t row = base + lane;
    const bool act = row < end;
    const uint32_t s = act ? slot[row] : 0u;
    const uint32_t v = act ? val[row] : 0u;
    const uint64_t actm = __ballot(act);
    if (VARIANT == 0) {
      if (act) atomicOr(reinterpret_cast<unsigned int*>(&tbl[s]) + (lane >> 5), 1u << (lane & 31));
      const uint64_t match = act ? tbl[s] : 0ull;
      const uint64_t below = match & lanes_below;
      const uint32_t lz = (uint32_t)__clzll((long long)below);
      const uint32_t pv = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(~lz << 2), (int)v);
      const bool diff = act && below != 0 && pv != v;
      const uint64_t dm = __ballot(diff);
      if (act && below == 0) {
        tbl[s] = 0ull;
        const State cur = st[s];
        const uint32_t rows = cur.rc & 0xFFFFu;
        uint32_t ch = (cur.rc >> 16) + (uint32_t)__popcll(dm & match);
        if (rows != 0 && cur.last != v) ch += 1u;
        if (rows == 0) ch += v != 0u ? 1u : 0u;  // zero-initialised last value
        st[s].rc = (rows + (uint32_t)__popcll(match)) | (ch << 16);
      }
      if (act && (match >> lane) == 1ull) st[s].last = v;
    } else {
      // stable LSD radix sort of (slot, lane) by slot; inactive lanes sort last (slot 511)
      uint32_t k = act ? s : (1u << kSlotBits) - 1u;
      uint32_t idx = (uint32_t)lane;
#pragma unroll
      for (int b = 0; b < kSlotBits; ++b) {
        const bool bit = (k >> b) & 1u;
        const uint64_t ones = __ballot(bit);
        const uint32_t nz = 64u - (uint32_t)__popcll(ones);
        const uint32_t dst = bit ? nz + mbcnt64(ones) : mbcnt64(~ones);
        k = (uint32_t)__builtin_amdgcn_ds_permute((int)(dst << 2), (int)k);
        idx = (uint32_t)__builtin_amdgcn_ds_permute((int)(dst << 2), (int)idx);
      }
      const uint32_t sv = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(idx << 2), (int)v);
      const bool sact = (actm >> idx) & 1ull;
      // previous sorted lane's slot and value (wave_shr:1; lane 0 reads the bound 0xFFFF...)
      const uint32_t pk = (uint32_t)__builtin_amdgcn_update_dpp((int)0xFFFFFFFF, (int)k, 0x138, 0xF, 0xF, false);
      const uint32_t pvv = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)sv, 0x138, 0xF, 0xF, false);
      const bool head = sact && (lane == 0 || pk != k);
      const uint64_t heads = __ballot(head);
      const uint64_t sactm = __ballot(sact);
      const bool diff = sact && !head && pvv != sv;
      const uint64_t dm = __ballot(diff);
      // the run of this head: lanes up to (not including) the next head, active lanes only
      const uint64_t after = lane == 63 ? 0ull : (heads >> (lane + 1)) << (lane + 1);
      const uint64_t upto = after ? ((after & (~after + 1ull)) - 1ull) : ~0ull;  // below the next head
      const uint64_t run = upto & ~lanes_below & sactm;
      if (head) {
        const State cur = st[k];
        const uint32_t rows = cur.rc & 0xFFFFu;
        uint32_t ch = (cur.rc >> 16) + (uint32_t)__popcll(dm & run);
        if (rows != 0 && cur.last != sv) ch += 1u;
        if (rows == 0) ch += sv != 0u ? 1u : 0u;
        st[k].rc = (rows + (uint32_t)__popcll(run)) | (ch << 16);
      }
      const bool tail = sact && (lane == 63 || ((heads >> (lane + 1)) & 1ull) || !((sactm >> (lane + 1)) & 1ull));
      if (tail) st[k].last = sv;
    }
  }
  __builtin_amdgcn_s_waitcnt(0xc07f);
  for (int i = lane; i < kSlots; i += 64) {
    atomicAdd(&out_rows[i], st[i].rc & 0xFFFFu);
    atomicAdd(&out_changes[i], st[i].rc >> 16);
  }
}

int main(int argc, char** argv) {
  const uint32_t n = argc > 1 ? (uint32_t)atoll(argv[1]) : 200u << 20;
  const int reps = argc > 2 ? atoi(argv[2]) : 20;
  std::vector<uint16_t> hs(n);
  std::vector<uint8_t> hv(n);
  uint64_t x = 88172645463325252ull;
  for (uint32_t i = 0; i < n; ++i) {
    x ^= x << 13; x ^= x >> 7; x ^= x << 17;
    hs[i] = (uint16_t)((x >> 8) % kSlots);
    hv[i] = (uint8_t)((x >> 40) % 10);
  }
  // host reference, chunk by chunk (a slot's state starts at zero in every chunk)
  std::vector<uint64_t> rrows(kSlots, 0), rch(kSlots, 0);
  for (uint32_t c0 = 0; c0 < n; c0 += kChunk) {
    std::vector<uint32_t> last(kSlots, 0), seen(kSlots, 0);
    for (uint32_t i = c0; i < std::min<uint64_t>(n, (uint64_t)c0 + kChunk); ++i) {
      const int s = hs[i];
      if (last[s] != hv[i]) ++rch[s];
      last[s] = hv[i];
      ++seen[s];
    }
    for (int s = 0; s < kSlots; ++s) rrows[s] += seen[s];
  }
  uint16_t* ds;
  uint8_t* dv;
  uint32_t* dout;
  CK(hipMalloc(&ds, (size_t)n * 2));
  CK(hipMalloc(&dv, n));
  CK(hipMalloc(&dout, 2 * kSlots * 4));
  CK(hipMemcpy(ds, hs.data(), (size_t)n * 2, hipMemcpyHostToDevice));
  CK(hipMemcpy(dv, hv.data(), n, hipMemcpyHostToDevice));
  const uint32_t waves = (n + kChunk - 1) / kChunk;
  const uint32_t blocks = (waves + kWaves - 1) / kWaves;
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int variant = 0; variant < 2; ++variant) {
    auto launch = [&]() {
      if (variant == 0) hipLaunchKernelGGL(k_match<0>, dim3(blocks), dim3(256), 0, 0, ds, dv, n, dout, dout + kSlots);
      else hipLaunchKernelGGL(k_match<1>, dim3(blocks), dim3(256), 0, 0, ds, dv, n, dout, dout + kSlots);
    };
    CK(hipMemset(dout, 0, 2 * kSlots * 4));
    launch();
    CK(hipDeviceSynchronize());
    std::vector<uint32_t> h(2 * kSlots);
    CK(hipMemcpy(h.data(), dout, h.size() * 4, hipMemcpyDeviceToHost));
    bool ok = true;
    for (int s = 0; s < kSlots; ++s) ok = ok && h[s] == rrows[s] && h[kSlots + s] == rch[s];
    CK(hipEventRecord(e0));
    for (int r = 0; r < reps; ++r) launch();
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    ms /= reps;
    printf("{\"variant\": \"%s\", \"rows\": %u, \"ms\": %.4f, \"GB_per_s\": %.1f, \"parity\": %s}\n",
           variant == 0 ? "lds_lane_masks" : "wave_counting_sort", n, ms, 3.0 * n / (ms * 1e6), ok ? "true" : "false");
    if (!ok) return 1;
  }
  return 0;
}
