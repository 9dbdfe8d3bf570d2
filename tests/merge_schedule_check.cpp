// Host check of the co-located merge's point-to-point schedules (bqueryd_amd/csrc/
// merge_schedule.h, the code comm.hip posts as grouped ncclSend / ncclRecv) -- TEST CODE,
// built and run by tests/test_merge_schedule.py with g++ (no GPU, no RCCL).
//
// For random count matrices (zero rows between some pairs, ranks that send or receive
// nothing) and column widths, every rank's exchange and gather lists are built exactly as
// comm.hip builds them; then, for every (sender, receiver) pair, the sender's messages to the
// receiver and the receiver's messages from the sender must agree one for one, in posting
// order, with equal byte counts (RCCL's matching rule).  The messages are then "delivered" in
// that order and every received element must be the one its sender packed for it, at the
// receiver's row offset for that sender.
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <random>
#include <vector>

#include "../bqueryd_amd/csrc/merge_schedule.h"

using bqg_sched::P2P;

static int fail(const char* what, int trial) {
  std::printf("FAIL trial %d: %s\n", trial, what);
  return 1;
}

// element value of (sender, receiver, column, row): what the receiver must find
static uint64_t tag(int s, int d, int j, int64_t row) {
  return ((uint64_t)s << 56) ^ ((uint64_t)d << 48) ^ ((uint64_t)j << 40) ^ (uint64_t)row ^ 0x5A5A5A5Aull;
}

static void put(unsigned char* p, int lg, int64_t i, uint64_t v) { std::memcpy(p + ((size_t)i << lg), &v, (size_t)1 << lg); }
static uint64_t get(const unsigned char* p, int lg, int64_t i) {
  uint64_t v = 0;
  std::memcpy(&v, p + ((size_t)i << lg), (size_t)1 << lg);
  return v;
}
static uint64_t trunc(uint64_t v, int lg) { return lg == 3 ? v : (v & ((1ull << (8 << lg)) - 1ull)); }

// deliver: for every (s, d) pair the posted lists must match one for one
static bool deliver(int W, const std::vector<std::vector<P2P>>& sends, const std::vector<std::vector<P2P>>& recvs) {
  for (int s = 0; s < W; ++s)
    for (int d = 0; d < W; ++d) {
      std::vector<const P2P*> a, b;
      for (const P2P& x : sends[s])
        if (x.peer == d) a.push_back(&x);
      for (const P2P& x : recvs[d])
        if (x.peer == s) b.push_back(&x);
      if (a.size() != b.size()) return false;
      for (size_t i = 0; i < a.size(); ++i) {
        if (a[i]->bytes != b[i]->bytes) return false;
        std::memcpy(b[i]->ptr, a[i]->ptr, a[i]->bytes);
      }
    }
  return true;
}

int main() {
  std::mt19937_64 rng(12345);
  for (int trial = 0; trial < 400; ++trial) {
    const int W = 1 + (int)(rng() % 9);
    const int ncols = 1 + (int)(rng() % 6);
    std::vector<int> lg(ncols);
    for (int& x : lg) x = (int)(rng() % 4);
    // count matrix C[s][d]: rows rank s sends to rank d (about a quarter of the pairs empty)
    std::vector<std::vector<int64_t>> C(W, std::vector<int64_t>(W));
    for (auto& row : C)
      for (int64_t& x : row) x = (rng() % 4 == 0) ? 0 : (int64_t)(rng() % 300);
    // sender side: rank s's packed rows for destination d, column j (the pack kernel's blocks)
    std::vector<std::vector<std::vector<std::vector<unsigned char>>>> sendbuf(W);
    for (int s = 0; s < W; ++s) {
      sendbuf[s].resize(W);
      for (int d = 0; d < W; ++d) {
        sendbuf[s][d].resize(ncols);
        for (int j = 0; j < ncols; ++j) {
          sendbuf[s][d][j].resize(((size_t)C[s][d] << lg[j]) + 8);
          for (int64_t r = 0; r < C[s][d]; ++r) put(sendbuf[s][d][j].data(), lg[j], r, tag(s, d, j, r));
        }
      }
    }
    // receiver side: one table of all rows received, sources in rank order
    std::vector<std::vector<std::vector<unsigned char>>> recvbuf(W);
    std::vector<std::vector<P2P>> sends(W), recvs(W);
    for (int r = 0; r < W; ++r) {
      std::vector<int64_t> to_peer(W), from_peer(W);
      int64_t total = 0;
      for (int x = 0; x < W; ++x) {
        to_peer[x] = C[r][x];
        from_peer[x] = C[x][r];
        total += from_peer[x];
      }
      recvbuf[r].resize(ncols);
      std::vector<void*> dst(ncols);
      for (int j = 0; j < ncols; ++j) {
        recvbuf[r][j].assign(((size_t)total << lg[j]) + 8, 0xEE);
        dst[j] = recvbuf[r][j].data();
      }
      bqg_sched::exchange_schedule(W, ncols, lg, to_peer, from_peer,
                                   [&](int d, int j) { return (void*)sendbuf[r][d][j].data(); }, dst, sends[r], recvs[r]);
    }
    if (!deliver(W, sends, recvs)) return fail("exchange: send / receive lists of a pair disagree", trial);
    for (int d = 0; d < W; ++d) {
      int64_t off = 0;
      for (int s = 0; s < W; ++s) {
        for (int j = 0; j < ncols; ++j)
          for (int64_t r = 0; r < C[s][d]; ++r)
            if (get(recvbuf[d][j].data(), lg[j], off + r) != trunc(tag(s, d, j, r), lg[j]))
              return fail("exchange: a received element is not the one its sender packed", trial);
        off += C[s][d];
      }
    }
    // gather: every rank's reduced partition (part_rows[r] rows) to rank 0, after its own
    std::vector<int64_t> part(W);
    int64_t gtotal = 0;
    for (int64_t& x : part) {
      x = (rng() % 5 == 0) ? 0 : (int64_t)(rng() % 500);
      gtotal += x;
    }
    std::vector<std::vector<std::vector<unsigned char>>> red(W);
    std::vector<std::vector<unsigned char>> root(ncols);
    std::vector<std::vector<P2P>> gs(W), gr(W);
    for (int j = 0; j < ncols; ++j) root[j].assign(((size_t)gtotal << lg[j]) + 8, 0xEE);
    for (int r = 0; r < W; ++r) {
      red[r].resize(ncols);
      std::vector<void*> src(ncols), dst(ncols, nullptr);
      for (int j = 0; j < ncols; ++j) {
        red[r][j].resize(((size_t)part[r] << lg[j]) + 8);
        for (int64_t i = 0; i < part[r]; ++i) put(red[r][j].data(), lg[j], i, tag(r, 0, j, i));
        src[j] = red[r][j].data();
        if (r == 0) {
          dst[j] = root[j].data();
          std::memcpy(root[j].data(), red[0][j].data(), (size_t)part[0] << lg[j]);  // rank 0's own rows
        }
      }
      bqg_sched::gather_schedule(r, W, ncols, lg, part, src, dst, gs[r], gr[r]);
    }
    if (!deliver(W, gs, gr)) return fail("gather: send / receive lists of a pair disagree", trial);
    int64_t off = 0;
    for (int s = 0; s < W; ++s) {
      for (int j = 0; j < ncols; ++j)
        for (int64_t i = 0; i < part[s]; ++i)
          if (get(root[j].data(), lg[j], off + i) != trunc(tag(s, 0, j, i), lg[j]))
            return fail("gather: a row is not at its rank's offset", trial);
      off += part[s];
    }
  }
  std::printf("OK\n");
  return 0;
}
