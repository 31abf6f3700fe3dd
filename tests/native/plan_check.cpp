// CPU check of the multi-GPU exchange bookkeeping (fm_spark_amd/csrc/fm_plan.h) that fm_group.hip
// runs on every rank: R simulated ranks each compute their own plans from the same all-gathered
// route counts, every element is tagged with (source, destination, index) and moved block by block
// the way a grouped ncclSend / ncclRecv pairs them, and each rank's receive buffer must then hold
// its sources' blocks in source order with every block's elements in order.  Covers the entry
// exchange (packed plan, from route_counts), the S-row exchange (requester -> owner, packed) and
// the chunked partial exchange (owner -> requester, chunk by chunk) for R = 1..9 and C = 1..7,
// blocks of zero included.
#include <cstdint>
#include <cstdio>
#include <random>
#include <vector>

#include "fm_plan.h"

using fmhip::plan::Plan;

static int failures = 0;
#define CHECK(c)                                                        \
  do {                                                                  \
    if (!(c)) {                                                         \
      std::printf("FAIL %s:%d: %s\n", __FILE__, __LINE__, #c);          \
      ++failures;                                                       \
    }                                                                   \
  } while (0)

struct Tag {
  int src, dst;
  int64_t idx;
};

// Rank r's send buffer for an exchange where it sends out[r][p] elements to p, blocks peer-major.
static std::vector<Tag> make_send(const std::vector<std::vector<int64_t>>& out, int r) {
  std::vector<Tag> b;
  for (size_t p = 0; p < out[r].size(); ++p)
    for (int64_t i = 0; i < out[r][p]; ++i) b.push_back({r, (int)p, i});
  return b;
}

// Move every (sender, receiver) block as RCCL would pair them; receive buffers sized by in-counts.
static void run(const std::vector<Plan>& pl, const std::vector<std::vector<Tag>>& send,
                std::vector<std::vector<Tag>>& recv) {
  const int R = (int)pl.size();
  for (int a = 0; a < R; ++a)
    for (int b = 0; b < R; ++b) {
      CHECK(pl[a].sc[b] == pl[b].rc[a]);  // a's send to b is b's receive from a
      if (pl[a].sc[b] != pl[b].rc[a]) continue;
      for (int64_t i = 0; i < pl[a].sc[b]; ++i) {
        const int64_t s = pl[a].so[b] + i, d = pl[b].ro[a] + i;
        CHECK(s >= 0 && s < (int64_t)send[a].size() && d >= 0 && d < (int64_t)recv[b].size());
        if (s >= 0 && s < (int64_t)send[a].size() && d >= 0 && d < (int64_t)recv[b].size()) recv[b][d] = send[a][s];
      }
    }
}

// recv[b] must be source-major blocks of in[b][s] elements, each from s to b, in index order.
static void expect_blocks(const std::vector<std::vector<Tag>>& recv, const std::vector<std::vector<int64_t>>& in) {
  for (size_t b = 0; b < recv.size(); ++b) {
    int64_t at = 0;
    for (size_t s = 0; s < in[b].size(); ++s)
      for (int64_t i = 0; i < in[b][s]; ++i, ++at) {
        const Tag& t = recv[b][at];
        CHECK(t.src == (int)s && t.dst == (int)b && t.idx == i);
      }
    CHECK(at == (int64_t)recv[b].size());
  }
}

int main() {
  std::mt19937_64 rng(20261017);
  int cases = 0;
  for (int R = 1; R <= 9; ++R) {
    for (int trial = 0; trial < 6; ++trial, ++cases) {
      // the job's route counts as ctx->sh_tot all-gathers them: [s][pairs to o (R) | entries to o (R)]
      std::vector<unsigned long long> all((size_t)R * 2 * R);
      for (int s = 0; s < R; ++s)
        for (int o = 0; o < R; ++o) {
          const bool empty = rng() % 5 == 0;  // blocks of zero
          const unsigned long long pairs = empty ? 0 : 1 + rng() % 40;
          const unsigned long long ents = pairs == 0 ? 0 : pairs + rng() % (3 * pairs + 1);  // >= 1 per pair
          all[(size_t)s * 2 * R + o] = pairs;
          all[(size_t)s * 2 * R + R + o] = ents;
        }
      std::vector<fmhip::plan::RouteCounts> rc;
      for (int r = 0; r < R; ++r) rc.push_back(fmhip::plan::route_counts(all.data(), R, r));
      std::vector<std::vector<int64_t>> eout(R), ein(R), pout(R), pin(R);
      for (int r = 0; r < R; ++r) {
        eout[r] = rc[r].ent_out;
        ein[r] = rc[r].ent_in;
        pout[r] = rc[r].pair_out;
        pin[r] = rc[r].pair_in;
        for (int o = 0; o < R; ++o) {  // route_counts is the transpose on the receiving side
          CHECK(rc[r].ent_out[o] == rc[o].ent_in[r]);
          CHECK(rc[r].pair_out[o] == rc[o].pair_in[r]);
        }
      }
      // entries: requester -> owner (packed)
      {
        std::vector<Plan> pl;
        std::vector<std::vector<Tag>> send(R), recv(R);
        for (int r = 0; r < R; ++r) {
          pl.push_back(fmhip::plan::packed(eout[r].data(), ein[r].data(), R));
          send[r] = make_send(eout, r);
          int64_t n = 0;
          for (int64_t v : ein[r]) n += v;
          recv[r].assign(n, Tag{-1, -1, -1});
        }
        run(pl, send, recv);
        expect_blocks(recv, ein);
      }
      // S rows: requester -> owner, one per pair (packed, pair counts)
      {
        std::vector<Plan> pl;
        std::vector<std::vector<Tag>> send(R), recv(R);
        for (int r = 0; r < R; ++r) {
          pl.push_back(fmhip::plan::packed(pout[r].data(), pin[r].data(), R));
          send[r] = make_send(pout, r);
          int64_t n = 0;
          for (int64_t v : pin[r]) n += v;
          recv[r].assign(n, Tag{-1, -1, -1});
        }
        run(pl, send, recv);
        expect_blocks(recv, pin);
      }
      // partial rows: owner -> requester, chunk by chunk; after all chunks the requester's buffer
      // is the packed result (owner-major blocks of its pair_out, pairs in order)
      for (int C = 1; C <= 7; ++C) {
        std::vector<std::vector<Tag>> send(R), recv(R);
        for (int r = 0; r < R; ++r) {
          send[r] = make_send(pin, r);  // the owner's partials: source-major, pair_in[q] rows for q
          int64_t n = 0;
          for (int64_t v : pout[r]) n += v;
          recv[r].assign(n, Tag{-1, -1, -1});
        }
        std::vector<int64_t> sent(R, 0);
        for (int c = 0; c < C; ++c) {
          std::vector<Plan> pl;
          for (int r = 0; r < R; ++r) pl.push_back(fmhip::plan::chunk(pin[r].data(), pout[r].data(), R, c, C));
          for (int r = 0; r < R; ++r)
            for (int q = 0; q < R; ++q) sent[r] += pl[r].sc[q];
          run(pl, send, recv);
        }
        for (int r = 0; r < R; ++r) {
          int64_t n = 0;
          for (int64_t v : pin[r]) n += v;
          CHECK(sent[r] == n);  // the chunks cover every partial row exactly once
        }
        expect_blocks(recv, pout);
      }
    }
  }
  std::printf("%d cases, %d failure(s)\n", cases, failures);
  return failures ? 1 : 0;
}
