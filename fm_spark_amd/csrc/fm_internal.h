// Internal declarations shared by the HIP translation units of libfm_hip.so.
// Nothing here crosses the C-ABI (include/fm_hip.h).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/fm_hip.h"

namespace fmhip {

// ------------------------------------------------------------------------ errors
void set_error(const std::string& msg);

struct Error {
  int code;
  std::string msg;
};

#define FM_HIP_CHECK(expr)                                                            \
  do {                                                                                \
    hipError_t _e = (expr);                                                           \
    if (_e != hipSuccess)                                                             \
      throw ::fmhip::Error{_e == hipErrorOutOfMemory ? FM_ERR_OOM : FM_ERR_HIP,        \
                           std::string(#expr) + ": " + hipGetErrorString(_e)};        \
  } while (0)

#define FM_REQUIRE(cond, msg)                                \
  do {                                                       \
    if (!(cond)) throw ::fmhip::Error{FM_ERR_ARG, (msg)};    \
  } while (0)

// -------------------------------------------------------------------- device table
// Per feature row, one record aligned to a 64- or 128-byte line so that a random row access
// costs one line (random gathers on MI355X are bound by 128-byte line requests):
//   float V[kp]          kp = roundup(k, 4); padding columns stay exactly 0 through updates
//   RowHdr {w, t, cum}   at float offset kp (16-byte aligned)
//   t   : epoch (executed steps) through which the row is current; -1 = absent
//   cum : sum of lambda over executed steps 1..t, i.e. the L1 shrink already applied.
// A row read at epoch E is brought current by S_{cum[E] - cum} (lazy L1, see fm_kernels.hip).
struct alignas(16) RowHdr {
  float w;
  int32_t t;
  double cum;
};

struct TableView {
  float* rec;      // [rows * stride]
  int64_t rows;    // local rows
  int32_t k;
  int32_t kp;
  int32_t stride;  // record stride in floats (16 or 32, or a multiple of 32)
  int32_t shard_count;
  int32_t shard_index;
  __host__ __device__ float* v(int64_t slot) const { return rec + slot * stride; }
  __host__ __device__ RowHdr* hdr(int64_t slot) const {
    return reinterpret_cast<RowHdr*>(rec + slot * stride + kp);
  }
};

// record stride (floats) for k factors: the smallest 64 B / 128 B line that holds V + header,
// else a multiple of 128 B
inline int32_t record_stride(int32_t kp) {
  const int32_t need = kp + 4;
  if (need <= 16) return 16;
  if (need <= 32) return 32;
  return (need + 31) / 32 * 32;
}

// device buffer helper
struct DevBuf {
  void* p = nullptr;
  size_t bytes = 0;
  void ensure(size_t n);
  // at least n bytes; a growth takes an eighth more (batches refilled with slightly different
  // sizes, e.g. randomSplit splits, then stop growing: a growth drains the device)
  void ensure_slack(size_t n) {
    if (n > bytes || !p) ensure(n + n / 8 + 4096);
  }
  void release();
  template <class T>
  T* as() const { return reinterpret_cast<T*>(p); }
};

// ------------------------------------------------------------------- radix sort
struct SortWork {
  DevBuf keys_a, keys_b, vals_a, vals_b, counts, digit_tot;
  int64_t cap = 0;
  void ensure(int64_t n);
};

// Stable LSD sort of (key, index) pairs: keys_in[n] (uint32, < 2^key_bits) with payload
// = original index (vals_in == nullptr) or vals_in[n].  Returns pointers to the sorted
// keys / payloads (inside `w`).
void radix_sort_pairs(SortWork& w, const uint32_t* keys_in, const uint32_t* vals_in, int64_t n,
                      int key_bits, hipStream_t st, const uint32_t** keys_out,
                      const uint32_t** vals_out);
// Same with an 8-byte payload (e.g. the exploded entry {sample, x}).  When final_keys /
// final_vals are given, the last pass writes there (a batch's own sorted view).
void radix_sort_pairs64(SortWork& w, const uint32_t* keys_in, const uint2* vals_in, int64_t n,
                        int key_bits, hipStream_t st, const uint32_t** keys_out,
                        const uint2** vals_out, uint32_t* final_keys = nullptr,
                        uint2* final_vals = nullptr);
// Stable sort by key bits [lo_bit, hi_bit) only (the bits below ride along), output written to
// final_keys / final_vals.
void radix_sort_pairs64_bits(SortWork& w, const uint32_t* keys_in, const uint2* vals_in, int64_t n, int lo_bit,
                             int hi_bit, hipStream_t st, uint32_t* final_keys, uint2* final_vals);

// ---------------------------------------------------------------- step kernels
// A device-resident mini-batch: the exploded (sampleId, featureId, featureValue) rows of
// Model.scala:148-153 kept both as CSR (row_ptr) and as COO entries ent[e] = {sample, x bits}.
struct BatchDev {
  int64_t n_rows = 0, nnz = 0;
  DevBuf row_ptr, col, ent, label;  // int64 [B+1], uint32 [N] feature slot, uint2 [N], double [B]
  DevBuf xs;                         // fp32 [N]: x alone, the forward's stream (8 B per entry with col)
};

// The single-table step's per-sample record: S (kp floats) and, for kp <= 16, the sample's
// {r, yhat} in the same 64-B (kp <= 12) or 128-B (kp = 16) record, so the update's S gather and
// {r, yhat} load hit one line; wider rows keep {r, yhat} in StepWork::yl.
inline bool s_rec_yl(int kp) { return kp <= 16; }
inline int s_rec_floats(int kp) { return s_rec_yl(kp) ? (kp + 2 <= 16 ? 16 : 32) : kp; }

struct StepWork {
  DevBuf S;         // [B * kp] float: per-sample vfxiSum
  DevBuf yl;        // [B] float2 {r, yhat}: r = yhat - y formed in fp64 from the fp64 label, then rounded
  DevBuf loss_part; // [n_fwd_blocks] double2 {loss, n_loss}
  DevBuf part;      // [ceil(N / 256) * 2 * (kp+2)] double partial gradients (one range per update wave)
  DevBuf ucnt;      // [n_update_blocks] uint32 distinct-id counts per block
  SortWork sort;
};

struct StepParams {
  int64_t n_rows;
  double eta;        // stepSize / sqrt(t)
  double lam;        // eta * regParam
  double scale_v;    // eta / m
  double m;          // miniBatchSize as double: (sum / m) * eta
  int32_t epoch;     // steps executed before this one (E)
  double cumE;       // cum[E]
  double cum_next;   // cum[E] + lam = cum[E+1]
  double w0;
};

// the forward's inference modes (fm_kernels.hip): 2 = predict (clamp bounds, fp64 score per
// sample into pred), 3 = calcLossGrad (fp64 pred / loss / dw per entry, dv [entries][k], the
// absent-id flag)
struct FwdOut {
  int mode = 0;
  double lo = 0.0, hi = 0.0;
  double* pred = nullptr;
  double* loss = nullptr;
  double* dw = nullptr;
  double* dv = nullptr;
  int32_t* absent = nullptr;
  uint32_t* pcount = nullptr;  // partial pass (sharded predict): present rows per pair
  // partial pass over chunk ch_c of ch_C (ch_C > 1): of every source r < ch_R, the pairs
  // [off[r] + P_r ch_c / ch_C, off[r] + P_r (ch_c + 1) / ch_C), P_r = off[r + 1] - off[r] (device off)
  const int64_t* ch_off = nullptr;
  int32_t ch_R = 0, ch_c = 0, ch_C = 1;
  // loss-grad mode: fill_sd > 0 gives an entry whose id the model lacks its own N(0, fill_sd^2)
  // w and v draws (calcLossGrad's coalesce with randn / udfInitVec, Model.scala:144-146,170-171),
  // keyed by (fill_seed, entry index, column)
  double fill_sd = 0.0;
  uint64_t fill_seed = 0;
  // train mode: the forward applies the update of every row whose header carries no multi tag of
  // this epoch (a singleton; fm_kernels.hip "Singleton rows"), with sp; kp <= 16
  bool fused = false;
  StepParams sp{};
};
constexpr int kMaxChunkSources = 64;  // sources a chunked partial pass can split
// partial_out != nullptr: the sharded owner's partial pass (fm_shard.hip): [pairs][kp] fp32 vectors
// followed by [pairs] float2 scalars (pred->pcount, if given: present rows per pair);
// else pred != nullptr: FactorizationMachinesModel.predict / calcLossGrad (p.w0, p.cumE used)
void launch_forward(const TableView& T, const BatchDev& b, StepWork& w, const StepParams& p,
                    hipStream_t st, int64_t* n_fwd_blocks, float* partial_out = nullptr,
                    const FwdOut* pred = nullptr);
// per-sample inputs of the segmented update: S rows of s_stride floats, {yhat, y} at yl[s * yl_stride]
struct SegSource {
  const float* S;
  int64_t s_stride;
  const float2* yl;
  int64_t yl_stride;
  // non-null: the entry count is n_dev[0] (device) <= N, and n_dev[1] singleton rows were updated
  // by the fused forward (added to the distinct count)
  const int64_t* n_dev = nullptr;
};
// emit != nullptr (replicated mode): the per-slot gradient sums go to emit[rows][kp + 4] as
// [sum g_V (kp) | sum g_w | 1 (touched) | 0] instead of being applied to the table
void launch_segment_update(const TableView& T, const BatchDev& b, StepWork& w, const StepParams& p,
                           const uint32_t* skeys, const uint2* sents, int64_t n_fwd_blocks,
                           double* stats_out, hipStream_t st, float* emit = nullptr, const int64_t* n_dev = nullptr);
// the fused step's singleton split of a prepared sorted view, at the step (fm_kernels.hip "Singleton
// rows"): the entries of runs of two or more, in order, into mkeys / ments (capacity N); n_out[0] =
// their count, n_out[1] = the number of singleton runs (device); each multi run's row in tag_T gets
// the epoch's multi tag
struct SplitWork {
  DevBuf cnt, off;
};
void launch_split(const uint32_t* skeys, const uint2* sents, int64_t N, SplitWork& sw, uint32_t* mkeys, uint2* ments,
                  int64_t* n_out, hipStream_t st, const TableView& tag_T, int32_t epoch);
void launch_segment_update(const TableView& T, int64_t N, const SegSource& src, StepWork& w, const StepParams& p,
                           const uint32_t* skeys, const uint2* sents, int64_t n_loss_blocks, double* stats_out,
                           hipStream_t st, float* emit = nullptr);
// replicated mode: apply the all-reduced gradient sums grad[rows][kp + 4] to every touched row;
// the number of touched rows -> *n_touched (device, fp64 stats slot), through per-block counts in
// blk_touched[kReplApplyBlocks]
constexpr int kReplApplyBlocks = 256 * 16;
void launch_repl_apply(const TableView& T, const float* grad, const StepParams& p, uint32_t* blk_touched,
                       double* n_touched, hipStream_t st);

void launch_init_random(const TableView& T, const int32_t* ids, int64_t n, int64_t id_begin,
                        uint64_t seed, double sd, int32_t epoch, double cumE, hipStream_t st);
void launch_load_rows(const TableView& T, const int32_t* ids, int64_t n, const double* w,
                      const double* V, int32_t epoch, double cumE, hipStream_t st);
void launch_flush(const TableView& T, int32_t epoch, double cumE, hipStream_t st);
void launch_gather_rows(const TableView& T, const int32_t* ids, int64_t n, double cumE, double* w, double* V,
                        int8_t* present, hipStream_t st);
void launch_table_reset(const TableView& T, hipStream_t st);
void launch_predict(const TableView& T, const BatchDev& b, double cumE, double w0, double lo, double hi,
                    double* pred, hipStream_t st);
void launch_init_entries(const TableView& T, const uint32_t* col, int64_t n, uint64_t seed, double sd,
                         int32_t epoch, double cumE, hipStream_t st);
void launch_loss_grad(const TableView& T, const BatchDev& b, double cumE, double w0, double* pred,
                      double* loss, double* dw, double* dv, int32_t* absent_flag, hipStream_t st,
                      double fill_sd = 0.0, uint64_t fill_seed = 0);
void launch_segment_sum(const uint32_t* skeys, const uint32_t* svals, int64_t n, const double* vecs,
                        int32_t k, uint32_t* run_index, int32_t* out_keys, double* out_sums,
                        int64_t* n_out_dev, hipStream_t st);
void launch_count_present(const TableView& T, int64_t* out, hipStream_t st);
// the uploaded CSR image (row_ptr, label, xoff, col with bit 31 = a value follows, the compact
// non-unit values) -> the device batch: row_ptr / label / col copied, ent[e] = {sample of e, x
// bits} rebuilt from row_ptr and the compact values (the explode of Model.scala:148-153)
void launch_explode(const int64_t* row_ptr_in, const double* label_in, const int32_t* xoff, const uint32_t* col_in,
                    const float* x_in, int64_t B, int64_t N, int64_t* row_ptr, double* label, uint32_t* col, uint2* ent,
                    float* xs, hipStream_t st);

// fm_batch_from_rows: dst row s = src row rows[s] (device rows[B]); row_ptr_in[B + 1] (device) is the
// result's row_ptr, computed by the host from the source's
void launch_select_rows(const BatchDev& src, const int64_t* rows, const int64_t* row_ptr_in, int64_t B, BatchDev& dst,
                        hipStream_t st);
// fm_batch_create_splits: each split's own row_ptr (rebased to its first entry) into split_rp
// [B + n_splits] and every entry's sample index made relative to its split's first row
// (split_rows [n_splits + 1], device)
void launch_split_rebase(const BatchDev& b, const int64_t* split_rows, int32_t n_splits, int64_t* split_rp,
                         hipStream_t st);

}  // namespace fmhip
