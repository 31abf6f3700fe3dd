// Host-side bookkeeping of the multi-GPU exchanges (fm_group.hip), kept free of HIP so that the
// CPU test suite can check it for any rank count (tests/native/plan_check.cpp): every rank computes
// its own plan from the job's all-gathered counts, and the plans of two ranks must agree on every
// block they exchange.
//
// Replaces the bookkeeping of the reference's shuffles S1/S2/S5/S6 (FactorizationMachinesModel.scala:
// 155-164, FactorizationMachinesSGD.scala:142-166): which entries and partial rows go to which rank,
// and where they land.
#pragma once

#include <cstdint>
#include <vector>

namespace fmhip {
namespace plan {

// One rank's all-to-all-v plan, in elements, per global peer p: send sc[p] elements from
// send + so[p] to p, receive rc[p] from p into recv + ro[p].
struct Plan {
  std::vector<int64_t> so, sc, ro, rc;
  explicit Plan(int R = 0) : so(R, 0), sc(R, 0), ro(R, 0), rc(R, 0) {}
};

// Packed all-to-all-v: blocks peer-major in both buffers; out[p] / in[p] elements to / from p.
inline Plan packed(const int64_t* out, const int64_t* in, int R) {
  Plan pl(R);
  int64_t so = 0, ro = 0;
  for (int p = 0; p < R; ++p) {
    pl.so[p] = so;
    pl.sc[p] = out[p];
    pl.ro[p] = ro;
    pl.rc[p] = in[p];
    so += out[p];
    ro += in[p];
  }
  return pl;
}

// Chunk c of C of the owners' partial exchange (fm_group.hip forward_exchange_chunked).  The owner
// sends the partial rows of the pair_in[q] pairs it received from requester q (laid out source-major);
// the requester receives them into its pair_out[o] block for owner o.  Chunk c of a block of P pairs
// is [P c / C, P (c + 1) / C) -- the same integer split on both sides, which the owner's kernel
// (shard_owner_partials) uses too.
inline Plan chunk(const int64_t* pair_in, const int64_t* pair_out, int R, int c, int C) {
  Plan pl(R);
  int64_t io = 0, oo = 0;
  for (int q = 0; q < R; ++q) {
    const int64_t Pi = pair_in[q], Po = pair_out[q];
    pl.so[q] = io + Pi * c / C;
    pl.sc[q] = Pi * (c + 1) / C - Pi * c / C;
    pl.ro[q] = oo + Po * c / C;
    pl.rc[q] = Po * (c + 1) / C - Po * c / C;
    io += Pi;
    oo += Po;
  }
  return pl;
}

// The job's route counts, all-gathered rank-major: all[s * 2R + o] = (sample, owner) pairs rank s
// sends owner o, all[s * 2R + R + o] = entries rank s sends owner o (ctx->sh_tot's layout) -> what
// rank gl sends (ent_out, pair_out: per owner) and receives (ent_in, pair_in: per source).
struct RouteCounts {
  std::vector<int64_t> ent_out, pair_out, ent_in, pair_in;
};
inline RouteCounts route_counts(const unsigned long long* all, int R, int gl) {
  RouteCounts rc;
  rc.ent_out.resize(R);
  rc.pair_out.resize(R);
  rc.ent_in.resize(R);
  rc.pair_in.resize(R);
  const unsigned long long* mine = all + (size_t)gl * 2 * R;
  for (int o = 0; o < R; ++o) {
    rc.pair_out[o] = (int64_t)mine[o];
    rc.ent_out[o] = (int64_t)mine[R + o];
  }
  for (int s = 0; s < R; ++s) {
    rc.pair_in[s] = (int64_t)all[(size_t)s * 2 * R + gl];
    rc.ent_in[s] = (int64_t)all[(size_t)s * 2 * R + R + gl];
  }
  return rc;
}

}  // namespace plan
}  // namespace fmhip
