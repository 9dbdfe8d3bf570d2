// blosc_micro.hip -- time k_blosc_decode on the splits of one blosc frame file (a raw blosc1
// frame, no bloscpack header): all splits together, and each non-raw split alone.
// build: hipcc -O3 -std=c++17 --offload-arch=gfx950 [-DBQG_BLOSC_PROF] -I bqueryd_amd/csrc
//        tools/micro/blosc_micro.hip -o build/blosc_micro
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "k_blosc.hip"  // one translation unit: the instrumentation symbols are file-local

#define CK(x)                                                              \
  do {                                                                     \
    hipError_t e_ = (x);                                                   \
    if (e_ != hipSuccess) {                                                \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      return 1;                                                            \
    }                                                                      \
  } while (0)

static int32_t le32(const unsigned char* p) {
  int32_t v;
  memcpy(&v, p, 4);
  return v;
}

int main(int argc, char** argv) {
  if (argc < 2) return 2;
  FILE* f = fopen(argv[1], "rb");
  if (!f) return 2;
  std::vector<unsigned char> fr;
  unsigned char buf[1 << 16];
  size_t n;
  while ((n = fread(buf, 1, sizeof buf, f)) > 0) fr.insert(fr.end(), buf, buf + n);
  fclose(f);
  const int reps = argc > 2 ? atoi(argv[2]) : 1;  // copies of the frame decoded together
  const unsigned flags = fr[2], ts = fr[3];
  const int64_t nbytes = le32(&fr[4]), bs = le32(&fr[8]), cb = le32(&fr[12]);
  const int64_t nblocks = (nbytes + bs - 1) / bs;
  printf("flags %#x ts %u nbytes %lld bs %lld cb %lld nblocks %lld\n", flags, ts, (long long)nbytes, (long long)bs,
         (long long)cb, (long long)nblocks);
  const size_t span = (fr.size() + 4095) & ~(size_t)4095;
  unsigned char *dcomp, *dout;
  unsigned int* bad;
  CK(hipMalloc(&dcomp, span * reps + bqg::kBloscPad));
  CK(hipMalloc(&dout, (size_t)nbytes * reps));
  CK(hipMalloc(&bad, 4));
  CK(hipMemset(bad, 0, 4));
  for (int r = 0; r < reps; ++r) CK(hipMemcpy(dcomp + r * span, fr.data(), fr.size(), hipMemcpyHostToDevice));
  std::vector<bqg::BloscSplit> all;
  for (int r = 0; r < reps; ++r)
    for (int64_t b = 0; b < nblocks; ++b) {
      const bool partial = b == nblocks - 1 && nbytes % bs;
      const int64_t bsize = partial ? nbytes % bs : bs;
      const int64_t ns = (!(flags & 0x10) && ts <= 16 && bs / ts >= 128 && !partial) ? ts : 1;
      int64_t p = le32(&fr[16 + 4 * b]);
      for (int64_t j = 0; j < ns; ++j) {
        const int64_t cs = le32(&fr[p]);
        p += 4;
        const int64_t ne = bsize / ns;
        all.push_back({(uint64_t)(r * span + p), (uint64_t)(dout + r * nbytes + b * bs + j * ne), (uint32_t)cs,
                       (uint32_t)ne, cs == ne ? bqg::kSplitRaw : (int32_t)(flags >> 5), 0});
        p += cs;
      }
    }
  bqg::BloscSplit* dt;
  CK(hipMalloc(&dt, all.size() * sizeof(bqg::BloscSplit)));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  auto run = [&](const std::vector<bqg::BloscSplit>& v, const char* what) -> int {
    CK(hipMemcpy(dt, v.data(), v.size() * sizeof(bqg::BloscSplit), hipMemcpyHostToDevice));
    bqg::launch_blosc_decode(dcomp, dt, (int)v.size(), bad, 0);  // warm
    CK(hipEventRecord(e0, 0));
    bqg::launch_blosc_decode(dcomp, dt, (int)v.size(), bad, 0);
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    uint64_t out = 0, comp = 0;
    for (auto& s : v) out += s.dsize, comp += s.csize;
    unsigned int hb;
    CK(hipMemcpy(&hb, bad, 4, hipMemcpyDeviceToHost));
#ifdef BQG_BLOSC_PROF
    if (v.size() == 1) {
      unsigned long long pr[32];
      CK(hipMemset(bad, 0, 4));
      unsigned long long z[32] = {};
      CK(hipMemcpyToSymbol(HIP_SYMBOL(bqg::g_blosc_prof), z, sizeof z));
      bqg::launch_blosc_decode(dcomp, dt, 1, bad, 0);
      CK(hipDeviceSynchronize());
      CK(hipMemcpyFromSymbol(pr, HIP_SYMBOL(bqg::g_blosc_prof), sizeof pr));
      const char* nm[8] = {"spec parse", "chain", "reparse+scan", "literals", "round tail", "round", "flush",
                           "serial seq"};
      for (int k = 0; k < 8; ++k)
        if (pr[16 + k]) printf("    %-12s n=%8llu  cycles/op %8.1f  total %.2f Mcyc\n", nm[k], pr[16 + k],
                               (double)pr[k] / pr[16 + k], pr[k] / 1e6);
    }
#endif
    printf("%-28s %6zu splits  %9.3f ms  %8.2f GB/s out  (comp %llu)  bad=%u\n", what, v.size(), ms,
           out / (ms * 1e6), (unsigned long long)comp, hb);
    return 0;
  };
  if (run(all, "all")) return 1;
  {
    // byte-exact check of every copy against <frame>.expect (the shuffled block bytes)
    std::string ep = std::string(argv[1]) + ".expect";
    FILE* fe = fopen(ep.c_str(), "rb");
    if (fe) {
      std::vector<unsigned char> ex((size_t)nbytes), got((size_t)nbytes * reps);
      const size_t rd = fread(ex.data(), 1, ex.size(), fe);
      fclose(fe);
      CK(hipMemcpy(got.data(), dout, got.size(), hipMemcpyDeviceToHost));
      size_t bad_bytes = 0, first = (size_t)-1;
      for (int r = 0; r < reps; ++r)
        for (size_t i = 0; i < ex.size(); ++i)
          if (got[(size_t)r * nbytes + i] != ex[i]) {
            if (first == (size_t)-1) first = (size_t)r * nbytes + i;
            ++bad_bytes;
          }
      printf("check vs %s (%zu bytes): %zu mismatches (first at %zd)\n", ep.c_str(), rd, bad_bytes,
             (ssize_t)first);
      if (bad_bytes) return 3;
    }
  }
  for (size_t i = 0; i < std::min<size_t>(all.size(), 16); ++i) {
    if (all[i].codec == bqg::kSplitRaw) continue;
    char name[64];
    snprintf(name, sizeof name, "split %zu alone", i);
    if (run({all[i]}, name)) return 1;
  }
  return 0;
}
