// Host check of bqueryd_amd/csrc/blosc_plan.h under -fsanitize=address,undefined (no GPU, no
// libblosc): the bcolz chunk-file parser that turns file bytes into the on-GPU decoder's
// stream tasks.  Well-formed frames (every flag / typesize / block-size shape the planner
// distinguishes) must plan into tasks that stay inside the file and the chunk's place in the
// column and cover the decoded bytes exactly; truncated, oversized and randomly corrupted
// files must come back as kError / kFallback or as tasks that still stay in bounds -- never as
// a read outside the file (each file sits in a heap block of exactly its size, so ASan sees any
// over-read).  Prints OK.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>
#include <vector>

#include "../bqueryd_amd/csrc/blosc_plan.h"

using namespace bqg;

static int failures = 0;
#define CHECK(c, ...)                          \
  do {                                         \
    if (!(c)) {                                \
      if (failures++ < 20) {                   \
        fprintf(stderr, "FAIL %s: ", #c);      \
        fprintf(stderr, __VA_ARGS__);          \
        fprintf(stderr, "\n");                 \
      }                                        \
    }                                          \
  } while (0)

static void put32(std::vector<unsigned char>& b, size_t at, int32_t v) { memcpy(&b[at], &v, 4); }

// A blosc1 frame as c-blosc 1.x lays it out: header, block offsets, per block `nsplits`
// streams {int32 csize, bytes}.  Stream bytes are filler (the planner does not decode).
static std::vector<unsigned char> make_file(std::mt19937_64& rng, int flags, int ts, int32_t nbytes, int32_t blocksize,
                                            bool raw_streams) {
  std::vector<unsigned char> f(kBloscpackHeader + kBloscHeader, 0);
  memcpy(f.data(), "blpk", 4);
  f[4] = 3;
  const size_t h = kBloscpackHeader;
  f[h + 0] = 2;
  f[h + 1] = 1;
  f[h + 2] = (unsigned char)flags;
  f[h + 3] = (unsigned char)ts;
  put32(f, h + 4, nbytes);
  put32(f, h + 8, blocksize);
  if (flags & 0x2) {  // memcpyed
    for (int32_t i = 0; i < nbytes; ++i) f.push_back((unsigned char)rng());
    put32(f, h + 12, (int32_t)(f.size() - h));
    return f;
  }
  const int64_t nblocks = nbytes ? (nbytes + blocksize - 1) / blocksize : 0;
  const int64_t leftover = nbytes % blocksize;
  const size_t table = f.size();
  f.resize(f.size() + 4 * (size_t)nblocks);
  for (int64_t b = 0; b < nblocks; ++b) {
    put32(f, table + 4 * b, (int32_t)(f.size() - h));
    const bool last_partial = b == nblocks - 1 && leftover != 0;
    const int64_t bsize = last_partial ? leftover : blocksize;
    const int64_t ns = (!(flags & 0x10) && ts <= 16 && blocksize / ts >= 128 && !last_partial) ? ts : 1;
    for (int64_t j = 0; j < ns; ++j) {
      const int32_t dsz = (int32_t)(bsize / ns);
      const int32_t csz = raw_streams ? dsz : (int32_t)(rng() % (dsz + 1));
      const size_t at = f.size();
      f.resize(f.size() + 4 + csz);
      put32(f, at, csz);
      for (int32_t k = 0; k < csz; ++k) f[at + 4 + k] = (unsigned char)rng();
    }
  }
  put32(f, h + 12, (int32_t)(f.size() - h));
  return f;
}

struct Outcome {
  Plan plan;
  std::vector<BloscSplit> splits;
  std::vector<BloscBlock> blocks;
};

// plan one file held in a heap block of exactly its size; check every task against the file
// and the chunk's output range
static Outcome plan_and_check(const std::vector<unsigned char>& bytes, size_t want, size_t chunk_bytes,
                              const char* what) {
  const size_t n = bytes.size();
  unsigned char* file = (unsigned char*)malloc(n ? n : 1);
  if (n) memcpy(file, bytes.data(), n);
  const uint64_t file_off = 4096, dst = 1ull << 40, tmp = 1ull << 41;
  ChunkFile cf{0, 7, file_off, n};
  Outcome o;
  std::string err;
  o.plan = plan_chunk(file, cf, dst, tmp, want, chunk_bytes, "test", o.splits, o.blocks, err);
  free(file);
  CHECK(o.plan != Plan::kError || !err.empty(), "%s: an error without a message", what);
  if (o.plan != Plan::kTasks) return o;
  uint64_t covered = 0;
  for (const BloscSplit& s : o.splits) {
    CHECK(s.src >= file_off + kBloscpackHeader && s.src + s.csize <= file_off + n,
          "%s: stream [%llu, +%u) outside the file [%llu, %llu)", what, (unsigned long long)s.src, s.csize,
          (unsigned long long)file_off, (unsigned long long)(file_off + n));
    const bool to_dst = s.dst >= dst && s.dst + s.dsize <= dst + want;
    const bool to_tmp = s.dst >= tmp && s.dst + s.dsize <= tmp + want;
    CHECK(to_dst || to_tmp, "%s: stream output [%llx, +%u) outside the chunk", what, (unsigned long long)s.dst, s.dsize);
    CHECK(s.codec == kSplitRaw || s.codec == kSplitBloscLz || s.codec == kSplitLz4, "%s: codec %d", what, s.codec);
    CHECK(s.codec != kSplitRaw || s.csize == s.dsize, "%s: a raw stream changes size", what);
    covered += s.dsize;
  }
  CHECK(covered == want, "%s: streams cover %llu of %zu bytes", what, (unsigned long long)covered, want);
  uint64_t shuffled = 0;
  for (const BloscBlock& b : o.blocks) {
    CHECK(b.dst >= dst && b.dst + b.bytes <= dst + want && b.tmp >= tmp && b.tmp + b.bytes <= tmp + want,
          "%s: shuffle block outside the chunk", what);
    // (a block need not be whole items: k_blosc_unshuffle copies the trailing bytes as they are,
    // like c-blosc's unshuffle)
    CHECK(b.typesize > 1, "%s: typesize %u", what, b.typesize);
    shuffled += b.bytes;
  }
  CHECK(o.blocks.empty() || shuffled == want, "%s: shuffle blocks cover %llu of %zu", what,
        (unsigned long long)shuffled, want);
  return o;
}

// 2. every truncation of the file: an error -- never a read past the end; 3. random
// corruption of the header, the offset table and the stream sizes.  Returns the errors seen.
static int abuse(std::mt19937_64& rng, const std::vector<unsigned char>& f, size_t nbytes, size_t chunk_bytes,
                 bool memcpyed) {
  int errors = 0;
  const size_t step = std::max<size_t>(1, f.size() / 97);
  for (size_t len = 0; len < f.size(); len += (len < 64 ? 1 : step)) {
    std::vector<unsigned char> t(f.begin(), f.begin() + len);
    Outcome q = plan_and_check(t, nbytes, chunk_bytes, "truncated");
    CHECK(q.plan != Plan::kTasks || nbytes == 0 || !memcpyed, "a truncated memcpyed frame planned (len %zu of %zu)",
          len, f.size());
    errors += q.plan == Plan::kError;
  }
  for (int m = 0; m < 60; ++m) {
    std::vector<unsigned char> c = f;
    const int kind = (int)(rng() % 5);
    const size_t hdr_end = std::min(c.size(), kBloscpackHeader + kBloscHeader + 64);
    if (kind == 0) {
      c[rng() % hdr_end] ^= (unsigned char)(1 + rng() % 255);
    } else if (kind == 1 && c.size() >= kBloscpackHeader + kBloscHeader) {
      const int32_t extremes[] = {0, -1, INT32_MIN, INT32_MAX, 15, 16, 17, (int32_t)c.size(), (int32_t)c.size() * 2};
      put32(c, kBloscpackHeader + 4 * (1 + rng() % 3), extremes[rng() % 9]);
    } else if (kind == 2 && c.size() >= 4) {
      const size_t at = rng() % (c.size() - 3);
      put32(c, at, (int32_t)rng());
    } else if (kind == 3) {
      for (int k = 0; k < 8; ++k) c[rng() % c.size()] = (unsigned char)rng();
    } else {
      c.resize(rng() % (c.size() + 1));
    }
    Outcome q = plan_and_check(c, nbytes, chunk_bytes, "corrupted");
    errors += q.plan == Plan::kError;
  }
  return errors;
}

int main(int argc, char** argv) {
  std::mt19937_64 rng(20261018);
  int planned = 0, fell_back = 0, errors = 0, real = 0;
  // 1. well-formed frames: codecs, shuffle on / off, typesizes, split / no-split, ragged last
  //    blocks, memcpyed frames, the empty frame
  const int codecs[] = {0 << 5, 1 << 5};
  const int tss[] = {1, 2, 4, 8, 16, 3, 24};
  for (int round = 0; round < 250; ++round) {
    const int ts = tss[rng() % 7];
    int flags = codecs[rng() % 2] | (rng() % 2 ? 0x1 : 0) | (rng() % 4 == 0 ? 0x10 : 0);
    if (rng() % 10 == 0) flags = 0x2;  // memcpyed
    const int32_t items = (int32_t)(rng() % 40000);
    const int32_t nbytes = items * ts;
    int32_t blocksize = (int32_t)((1 + rng() % 64) * 1024) / ts * ts;
    if (blocksize <= 0) blocksize = ts;
    const bool raw = rng() % 3 == 0;
    auto f = make_file(rng, flags, ts, nbytes, blocksize, raw);
    const size_t chunk_bytes = (size_t)nbytes + (rng() % 2 ? 0 : (size_t)ts * (rng() % 100));
    Outcome o = plan_and_check(f, (size_t)nbytes, chunk_bytes, "well-formed");
    CHECK(o.plan == Plan::kTasks || (flags & 0x10) || ts == 24 || ts == 3,
          "well-formed frame (flags %x ts %d nbytes %d blocksize %d) not planned", flags, ts, nbytes, blocksize);
    planned += o.plan == Plan::kTasks;
    fell_back += o.plan == Plan::kFallback;
    // a padded last frame (more bytes than the chunk's rows): the host fallback copies `want`
    if (nbytes > ts) {
      Outcome p = plan_and_check(f, (size_t)nbytes - ts, chunk_bytes, "padded");
      CHECK(p.plan == Plan::kFallback, "a frame larger than the rows it holds must fall back");
    }
    errors += abuse(rng, f, (size_t)nbytes, chunk_bytes, (flags & 0x2) != 0);
  }
  // 5. frames the system libblosc wrote (tests/test_blosc_plan.py), each as a bcolz chunk file
  for (int a = 1; a < argc; ++a) {
    FILE* fp = fopen(argv[a], "rb");
    if (!fp) {
      fprintf(stderr, "cannot read %s\n", argv[a]);
      return 2;
    }
    std::vector<unsigned char> f;
    unsigned char buf[65536];
    size_t got;
    while ((got = fread(buf, 1, sizeof(buf), fp)) > 0) f.insert(f.end(), buf, buf + got);
    fclose(fp);
    int32_t nbytes = 0;
    if (f.size() >= kBloscpackHeader + kBloscHeader) memcpy(&nbytes, &f[kBloscpackHeader + 4], 4);
    Outcome o = plan_and_check(f, (size_t)nbytes, (size_t)nbytes, argv[a]);
    CHECK(o.plan != Plan::kError, "%s: a libblosc frame did not plan", argv[a]);
    real += o.plan == Plan::kTasks;
    errors += abuse(rng, f, (size_t)nbytes, (size_t)nbytes, f[kBloscpackHeader + 2] & 0x2);
  }
  // 4. garbage files of every small size
  for (int round = 0; round < 3000; ++round) {
    std::vector<unsigned char> g(rng() % 200);
    for (auto& x : g) x = (unsigned char)rng();
    if (g.size() >= 4 && rng() % 2) memcpy(g.data(), "blpk", 4);
    plan_and_check(g, (size_t)(rng() % 1000), 1000 + rng() % 1000, "garbage");
  }
  CHECK(planned > 200 && errors > 1000, "coverage: %d planned, %d fell back, %d errors", planned, fell_back, errors);
  CHECK(argc == 1 || real > 0, "no libblosc frame planned into device tasks");
  if (failures) {
    fprintf(stderr, "%d failures\n", failures);
    return 1;
  }
  printf("OK\n");
  return 0;
}
