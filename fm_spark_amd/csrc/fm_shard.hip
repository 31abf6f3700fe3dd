// Sharded (row-partitioned) step entry points.  Placeholder until the exchange kernels land.
#include "fm_internal.h"

extern "C" {
int fm_shard_plan(fm_ctx*, const fm_batch*, int64_t*) { fmhip::set_error("sharded step not built yet"); return FM_ERR_STATE; }
int fm_shard_request_copy(fm_ctx*, void*) { fmhip::set_error("sharded step not built yet"); return FM_ERR_STATE; }
int fm_shard_serve_device(fm_ctx*, const void*, int64_t, void*) { fmhip::set_error("sharded step not built yet"); return FM_ERR_STATE; }
int fm_shard_local_grad_device(fm_ctx*, const fm_batch*, const void*, void*, int64_t) { fmhip::set_error("sharded step not built yet"); return FM_ERR_STATE; }
int fm_shard_apply_device(fm_ctx*, const void*, const void*, int64_t, int32_t, double, double, int64_t) { fmhip::set_error("sharded step not built yet"); return FM_ERR_STATE; }
int fm_shard_last_loss(fm_ctx*, double*, int64_t*) { fmhip::set_error("sharded step not built yet"); return FM_ERR_STATE; }
}
