// PyTorch bindings for the Perceiver IO CDNA4 kernels.  Host-only translation unit
// (g++): validates shapes/dtypes, allocates outputs, and launches on the current HIP
// stream so every call is capturable in a hipGraph.
#include <torch/extension.h>
#include <ATen/hip/HIPContext.h>
#include <hip/hip_runtime.h>

#include "pe_args.h"

#include <unordered_map>
#include <vector>

namespace pio {
struct AttnArgs {
  const uint16_t* q; long long q_bs; int q_rs;
  const uint16_t* k; long long k_bs; int k_rs;
  const uint16_t* v; long long v_bs; int v_rs;
  const uint8_t* kmask;
  int B, H, Nq, Nk;
  float scale_log2, scale;
  uint32_t drop_thresh;
  float drop_scale;
  const int64_t* seedp;
  uint32_t site;
};
struct DropCfg {  // common.h
  const int64_t* seed;
  uint32_t site;
  uint32_t thresh;
  float scale;
};
struct PostAttnGrads { float *dWo, *dbo, *dg2, *dbe2, *dW1, *db1, *dW2, *db2; int vrs; int slab; };
constexpr int kMaxSlabSegs = 16, kSlabColsPerBlock = 1024;  // common.h
struct SlabJob {
  const float* slab;
  int S, P, nbx, nblk;
  int det;
  int n;
  float* dst[kMaxSlabSegs];
  int off[kMaxSlabSegs];
  int len[kMaxSlabSegs];
  float* zero_p;  // (mirror of csrc/common.h)
  long long zero_n4;
};
}  // namespace pio
#include "persist_args.h"
#include "sb_args.h"
namespace pio {
bool sb_fwd_launch(const SBFwdArgs&, int C, hipStream_t);
bool sb_bwd_launch(const SBBwdArgs&, int C, hipStream_t);
bool sb_wgrad_launch(SBWgradArgs, int C, const SlabJob&, hipStream_t);
bool sa_block_fwd_launch(const SABlockFwdArgs&, hipStream_t);
unsigned persist_errors(bool);
void persist_set_spin_limit(unsigned);
int persist_sync_words(int);

// sizes of the structs above as the kernel translation units see them (checked at import: a
// mirror that drifts from common.h / attention.hip would hand the kernels garbage pointers)
int abi_struct_size(int which);
void attn_fwd_launch(const AttnArgs&, int, uint16_t*, float*, float*, float*, int, hipStream_t);
void attn_bwd_launch(const AttnArgs&, int, const uint16_t*, const uint16_t*, const float*, float*, float*, long long,
                     int, float*, long long, int, float*, long long, int, bool, bool, long long, int, int, hipStream_t);
int attn_bwd_key_blocks(int, int);
bool attn_bwd_bf16_ok(const AttnArgs&, int);
bool attn_bwd_bf16_launch(const AttnArgs&, int, const uint16_t*, const float*, const float*, uint16_t*, long long, int,
                          uint16_t*, long long, int, uint16_t*, long long, int, const SlabJob&, hipStream_t);
int attn_bwd_zero_plan(int, int, int, int, int);
void ln_linear_fwd_launch(const void*, bool, int, int, int, const float*, const float*, float, const uint16_t*, int,
                          const float*, int, int, const float*, int, void*, bool, int, float*, float*, const float*, int,
                          int, int, const long long*, hipStream_t);
void post_attn_fwd_launch(int, const uint16_t*, const float*, const uint16_t*, const float*, const float*,
                          const float*, float, const uint16_t*, const float*, const uint16_t*, const float*, float*,
                          float*, float*, float*, uint16_t*, int, int, const DropCfg&, hipStream_t);
void post_attn_ln_linear_fwd_launch(int, const uint16_t*, const float*, const uint16_t*, const float*, const float*,
                                    const float*, float, const uint16_t*, const float*, const uint16_t*, const float*,
                                    float*, float*, float*, float*, uint16_t*, int, int, const float*, const float*,
                                    const uint16_t*, const float*, uint16_t*, float*, float*, const DropCfg&,
                                    hipStream_t);
bool sa_layer_fwd_launch(const uint16_t*, int, float, uint16_t*, float*, const float*, const uint16_t*, const float*,
                         const float*, const float*, float, const uint16_t*, const float*, const uint16_t*, const float*,
                         float*, float*, float*, float*, uint16_t*, int, const float*, const float*, const uint16_t*,
                         const float*, uint16_t*, float*, float*, const DropCfg&, int, hipStream_t);
bool ln_linear_post_attn_bwd_launch(int, const void*, bool, const uint16_t*, const float*, const float*, const float*,
                                    const float*, const float*, const float*, float*, float*, float*, float*,
                                    const float*, const float*, const float*, const uint16_t*, const uint16_t*,
                                    const uint16_t*, const uint16_t*, const uint16_t*, const float*, const float*,
                                    float*, uint16_t*, float*, int, const PostAttnGrads&, int, const SlabJob&,
                                    const DropCfg&, int, const uint16_t*, const float*, uint16_t*, float, hipStream_t);
void post_attn_bwd_launch(int, const float*, const float*, const float*, const float*, const uint16_t*,
                          const uint16_t*, const uint16_t*, const uint16_t*, const uint16_t*, const float*,
                          const float*, float*, uint16_t*, float*, int, const PostAttnGrads&, int, const SlabJob&,
                          const DropCfg&, hipStream_t);
void ln_linear_bwd_launch(const void*, bool, int, int, const uint16_t*, int, int, const void*, bool, int, const float*,
                          const float*, const float*, const float*, const float*, int, float*, int, float*, float*,
                          float*, float*, int, int, int, int, const float*, int, int, int, const long long*, const SlabJob&,
                          hipStream_t);
void wgrad_launch(const void*, bool, int, int, const void*, bool, int, int, int, const float*, const float*,
                  const float*, const float*, int, int, float*, float*, int, int, const float*, int, int, int,
                  const long long*, hipStream_t);
void ce_fwd_launch(int, const float*, const int64_t*, const int64_t*, const uint16_t*, const float*, int, int, float*,
                   float*, float*, float*, float*, float*, unsigned*, uint16_t*, int, float*, long long, int, hipStream_t);
int ce_combine_blocks(int);
int ce2_num_splits(int, int);
int ce2_bwd_splits(int, int);
int ce2_row_blocks(int);
void ce2_fwd_launch(const float*, const int64_t*, const int64_t*, const uint16_t*, const float*, int, int, int, float2*,
                    float*, float*, uint16_t*, float*, float*, int, float*, float*, unsigned*, unsigned*, float*,
                    long long, hipStream_t);
void ce2_bwd_launch(const uint16_t*, const int64_t*, const uint16_t*, const float*, const float*, const float*,
                    const float2*, int, const float*, const float*, int, int, float*, float*, float*, int, float*, long long,
                    const int64_t*, hipStream_t);
int ce_num_splits(int, int);
int ce_dw_splits(int, int);
void mlm_select_launch(const int64_t*, int, int, int, int, int64_t*, int64_t*, int*, int64_t*, int64_t*, float*, bool*, bool*,
                       const float*, int, float*, hipStream_t);
void ce_bwd_launch(int, const uint16_t*, const int64_t*, const uint16_t*, const float*, const float*, const float*,
                   const float*, int, int, float*, long long, const int64_t*, float*, float*, int, float*, int, hipStream_t);
void embed_fwd_launch(const int64_t*, const float*, const float*, float*, long long, int, int, float, long long,
                      hipStream_t);
unsigned check_errors_elementwise(bool);
unsigned check_errors_mlm_head(bool);
unsigned check_errors_ce_head(bool);
unsigned check_errors_rowgemm(bool);
void embed_bwd_launch(const int64_t*, const float*, float*, float*, int, int, int, float, hipStream_t);
void embed_bwd_sorted_launch(const int64_t*, const int64_t*, const float*, float*, long long, int, float, hipStream_t);
bool embed_bwd_local_launch(const int64_t*, const float*, float*, float*, int, int, int, float, const SlabJob&,
                            hipStream_t);
void text_mask_launch(const int64_t*, const bool*, int64_t*, int64_t*, int64_t*, long long, int, int, float, int,
                      uint32_t, int, hipStream_t);
int stage_step_launch(void* const*, const void* const*, const long long*, int, float*, const float*, int, long long*,
                      const long long*, int, hipStream_t);
void sumsq_launch(const float*, long long, float*, hipStream_t);
void index_add_rows_launch(float*, long long, const int64_t*, const float*, long long, int, hipStream_t);
void gather_rows_launch(float*, const float*, long long, const int64_t*, long long, int, hipStream_t);
void batch_sum2_launch(const float*, const float*, float*, float*, int, long long, long long, int, hipStream_t);
void pe_gemm_launch(const uint16_t*, const uint16_t*, void*, bool, int, int, int, int, hipStream_t);
struct PeGradTargets { float *dWa, *dWb, *db, *dg, *dbeta; };
int pe_grad_splits(int);
void pe_grads_launch(const uint16_t*, const float*, int, int, int, const float*, int, float*, float*, float*,
                     const float*, const float*, const float*, const float*, int, int, int, PeGradTargets, hipStream_t);
void pe_weight_prep_launch(const float*, const float*, int, const float*, const float*, const float*, int, int, int, int,
                           uint16_t*, float*, float*, float*, float*, hipStream_t);
int pixel_ce_blocks(long long);
void pixel_ce_fwd_launch(int, int, const float*, const float*, const float*, const int64_t*, const float*, long long,
                         float*, float*, float*, hipStream_t);
void pixel_ce_bwd_launch(int, int, const float*, const float*, const float*, const int64_t*, const float*,
                         const float*, const float*, long long, float*, float*, float*, float*, hipStream_t);
void adamw_launch(float*, float*, float*, float*, uint16_t*, long long, const float*, float, float, float, float,
                  int, int, const float*, float*, int, const float*, hipStream_t);
void cast_bf16_launch(const float*, uint16_t*, long long, hipStream_t);
void reduce_probe_launch(const float*, float*, hipStream_t);
void fold_replicas_launch(float*, float*, long long, int, hipStream_t);
void slab_reduce_launch(const SlabJob&, hipStream_t);
void pe_proj_fwd_launch(const float*, int, const float*, const float*, const float*, const float*, const float*,
                        const float*, long long, int, int, int, float, uint16_t*, float*, float*, hipStream_t);
int pe_proj_bwd_blocks(int);
void attn_fwd_pe_launch(const PeFwdArgs&, hipStream_t);
int attn_fwd_pe_auto_splits(int, int, int);
void attn_combine_launch(const float*, const float*, uint16_t*, float*, int, long long, int, hipStream_t);
void attn_bwd_pe_launch(const PeBwdArgs&, int, int, hipStream_t);
void pe_proj_bwd_launch(const float*, const float*, int, const float*, const float*, int, int, int, float*, float*,
                        hipStream_t);
}  // namespace pio

using torch::Tensor;
using OptT = c10::optional<Tensor>;

namespace {
hipStream_t stream() { return at::hip::getCurrentHIPStream(); }

#ifndef PIO_CHECKS
#define PIO_CHECKS 0
#endif
// checked builds: the device error words of every checked translation unit (bit 1: a token id
// outside the embedding table, 2: a gather row outside its destination, 4: a class label
// outside [0, V) ∪ {-100}); reset clears them
int64_t check_errors(bool reset) {
  return (int64_t)(pio::check_errors_elementwise(reset) | pio::check_errors_mlm_head(reset) |
                   pio::check_errors_ce_head(reset) | pio::check_errors_rowgemm(reset));
}
bool checked_build() { return PIO_CHECKS != 0; }
// checked builds, outside graph capture: wait for the kernel just launched and raise on any
// device-side index violation (the kernel itself clamped / skipped the access)
void checked_sync(const char* what) {
  if (!PIO_CHECKS) return;
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  (void)hipStreamIsCapturing(stream(), &cs);
  if (cs != hipStreamCaptureStatusNone) return;
  (void)hipStreamSynchronize(stream());
  const int64_t e = check_errors(true);
  TORCH_CHECK(e == 0, "checked build: ", what, " saw out-of-range indices (error bits ", e,
              ": 1 token id >= vocab, 2 gather row out of range, 4 label outside [0, V) and != -100, 8 PE row index outside "
              "the position-encoding table)");
}

// deterministic mode (trainer flag ``deterministic``): every reduction that would
// use fp32 atomics with several writers per address runs as a fixed-order split reduction
bool g_det = false;

#define CHECK_CUDA(t) TORCH_CHECK((t).is_cuda(), #t " must be a GPU tensor")
#define CHECK_DT(t, dt) TORCH_CHECK((t).scalar_type() == (dt), #t " has wrong dtype ", (t).scalar_type())

const uint16_t* bfp(const Tensor& t) { CHECK_DT(t, torch::kBFloat16); return reinterpret_cast<const uint16_t*>(t.data_ptr()); }
uint16_t* bfp_mut(Tensor& t) { CHECK_DT(t, torch::kBFloat16); return reinterpret_cast<uint16_t*>(t.data_ptr()); }
const float* f32p(const Tensor& t) { CHECK_DT(t, torch::kFloat32); return t.data_ptr<float>(); }
const float* f32o(const OptT& t) { return t.has_value() ? f32p(*t) : nullptr; }
bool is_bf16(const Tensor& t) {
  TORCH_CHECK(t.scalar_type() == torch::kBFloat16 || t.scalar_type() == torch::kFloat32, "expected bf16/fp32");
  return t.scalar_type() == torch::kBFloat16;
}

// 3-D (B|1, N, >=HD) view with unit inner stride → (batch stride, row stride)
void strides3(const Tensor& t, int B, long long& bs, int& rs) {
  TORCH_CHECK(t.dim() == 3 && t.stride(2) == 1, "attention operand must be 3-D with unit inner stride");
  TORCH_CHECK(t.size(0) == B || t.size(0) == 1, "batch mismatch");
  bs = t.size(0) == 1 ? 0 : t.stride(0);
  rs = (int)t.stride(1);
  TORCH_CHECK(rs % 8 == 0 && (bs % 8 == 0) && (reinterpret_cast<uintptr_t>(t.data_ptr()) % 16 == 0),
              "attention operands need 16-byte aligned rows");
}

// device dropout seed: a 1-element int64 GPU tensor (drawn per forward call, see common.h DropCfg)
const int64_t* seed_ptr(const OptT& seed, double p) {
  if (!(p > 0)) return nullptr;
  TORCH_CHECK(seed.has_value(), "dropout > 0 needs a device seed tensor");
  TORCH_CHECK(seed->is_cuda() && seed->scalar_type() == torch::kInt64 && seed->numel() >= 1,
              "dropout seed must be an int64 GPU tensor");
  return seed->data_ptr<int64_t>();
}

pio::DropCfg make_drop(const OptT& seed, int64_t site, double p) {
  TORCH_CHECK(p >= 0 && p < 1, "dropout probability must be in [0, 1)");
  pio::DropCfg d{};
  d.seed = seed_ptr(seed, p);
  d.site = (uint32_t)site;
  d.thresh = p > 0 ? (uint32_t)std::min(4294967295.0, p * 4294967296.0) : 0u;
  d.scale = p > 0 ? (float)(1.0 / (1.0 - p)) : 1.f;
  return d;
}

pio::AttnArgs make_args(const Tensor& q, const Tensor& k, const Tensor& v, const OptT& kmask, int H, int D,
                        double scale, double dropout_p, const OptT& seed, int64_t site) {
  CHECK_CUDA(q); CHECK_CUDA(k); CHECK_CUDA(v);
  pio::AttnArgs a{};
  a.B = (int)std::max(q.size(0), k.size(0));
  a.H = H;
  a.Nq = (int)q.size(1);
  a.Nk = (int)k.size(1);
  TORCH_CHECK(v.size(1) == a.Nk, "K/V length mismatch");
  TORCH_CHECK(D == 16 || D == 32 || D == 64 || D == 128, "head dim must be 16/32/64/128, got ", D);
  TORCH_CHECK(q.size(2) >= H * D && k.size(2) >= H * D && v.size(2) >= H * D, "head columns out of range");
  TORCH_CHECK(k.size(0) == a.B && v.size(0) == a.B, "K/V must carry the full batch");
  a.q = bfp(q); a.k = bfp(k); a.v = bfp(v);
  strides3(q, a.B, a.q_bs, a.q_rs);
  strides3(k, a.B, a.k_bs, a.k_rs);
  strides3(v, a.B, a.v_bs, a.v_rs);
  a.kmask = nullptr;
  if (kmask.has_value()) {
    const Tensor& m = *kmask;
    CHECK_CUDA(m);
    TORCH_CHECK(m.scalar_type() == torch::kBool || m.scalar_type() == torch::kUInt8, "key mask must be bool/uint8");
    TORCH_CHECK(m.is_contiguous() && m.size(0) == a.B && m.size(1) == a.Nk, "key mask must be (B, Nk) contiguous");
    a.kmask = reinterpret_cast<const uint8_t*>(m.data_ptr());
  }
  a.scale = (float)scale;
  a.scale_log2 = (float)(scale * 1.4426950408889634);
  const pio::DropCfg d = make_drop(seed, site, dropout_p);
  a.drop_thresh = d.thresh;
  a.drop_scale = d.scale;
  a.seedp = d.seed;
  a.site = d.site;
  return a;
}
}  // namespace

std::vector<Tensor> attn_fwd(Tensor q, Tensor k, Tensor v, OptT kmask, int64_t H, int64_t D, double scale,
                             double dropout_p, OptT seed, int64_t nsplit, int64_t site) {
  auto a = make_args(q, k, v, kmask, (int)H, (int)D, scale, dropout_p, seed, site);
  auto opts = q.options();
  Tensor O = torch::empty({a.B, a.Nq, H * D}, opts.dtype(torch::kBFloat16));
  Tensor L = torch::empty({a.B, a.Nq, H}, opts.dtype(torch::kFloat32));
  Tensor Op, ML;
  float* opp = nullptr; float* mlp = nullptr;
  if (nsplit > 1) {
    Op = torch::empty({nsplit, a.B, a.Nq, H, D}, opts.dtype(torch::kFloat32));
    ML = torch::empty({nsplit, a.B, a.Nq, H, 2}, opts.dtype(torch::kFloat32));
    opp = Op.data_ptr<float>(); mlp = ML.data_ptr<float>();
  }
  pio::attn_fwd_launch(a, (int)D, bfp_mut(O), L.data_ptr<float>(), opp, mlp, (int)std::max<int64_t>(1, nsplit), stream());
  return {O, L};
}

// returns (dq, dk, dv) fp32; dq is per batch even when q is batch-broadcast.  Optional
namespace {
pio::SlabJob make_job(const OptT& slab, std::vector<Tensor>& dsts, const std::vector<int64_t>& offs);
}  // namespace

// *_out tensors (B, N, >=HD views, unit inner stride) let the results land in packed buffers;
// a dq_out view must be batch-dense (batch stride == Nq * row stride); it needs no zero fill
// (the launcher clears it itself when several key blocks accumulate into it).  delta_in ((B, Nq, H) fp32 rowsum(dO∘O), e.g. from post_attn_bwd)
// skips the delta pass.
std::vector<Tensor> attn_bwd(Tensor q, Tensor k, Tensor v, OptT kmask, Tensor o, Tensor dO, Tensor lse, OptT delta_in,
                             int64_t H, int64_t D, double scale, double dropout_p, OptT seed, OptT dq_out,
                             OptT dk_out, OptT dv_out, bool kv_accumulate, int64_t site, bool dq_zeroed,
                             bool kv_zeroed, OptT job_slab, std::vector<Tensor> job_dsts, std::vector<int64_t> job_offs) {
  auto a = make_args(q, k, v, kmask, (int)H, (int)D, scale, dropout_p, seed, site);
  // job (optional): the previous kernel's slab reduction, carried by the bf16 variant (else a
  // standalone launch first)
  const pio::SlabJob job = make_job(job_slab, job_dsts, job_offs);
  TORCH_CHECK(dO.is_contiguous() && o.is_contiguous(), "O / dO must be contiguous (B, Nq, H*D)");
  auto f32 = q.options().dtype(torch::kFloat32);
  if (dq_out.has_value() && dq_out->scalar_type() == torch::kBFloat16) {
    // bf16 outputs (all three, stored once each): the self-attention backward feeding the
    // chain-layout layer-boundary kernel, which reads them as bf16 operands
    TORCH_CHECK(dk_out.has_value() && dv_out.has_value() && dk_out->scalar_type() == torch::kBFloat16 &&
                    dv_out->scalar_type() == torch::kBFloat16 && delta_in.has_value() && !kv_accumulate,
                "bf16 attn_bwd outputs: dq/dk/dv all bf16, delta given, no accumulation");
    Tensor dq = *dq_out, dk = *dk_out, dv = *dv_out;
    TORCH_CHECK(dq.stride(2) == 1 && dk.stride(2) == 1 && dv.stride(2) == 1, "dq/dk/dv need unit inner stride");
    Tensor delta = *delta_in;
    TORCH_CHECK(delta.is_contiguous() && delta.numel() == (int64_t)a.B * a.Nq * H, "delta must be (B, Nq, H)");
    CHECK_DT(delta, torch::kFloat32);
    if (pio::attn_bwd_bf16_ok(a, (int)D)) {
      pio::attn_bwd_bf16_launch(a, (int)D, bfp(dO), f32p(lse), delta.data_ptr<float>(), bfp_mut(dq), dq.stride(0),
                                (int)dq.stride(1), bfp_mut(dk), dk.stride(0), (int)dk.stride(1), bfp_mut(dv),
                                dv.stride(0), (int)dv.stride(1), job, stream());
    } else {  // shape not covered by the bf16 variant: fp32, then narrowed
      if (job.slab) pio::slab_reduce_launch(job, stream());
      std::vector<Tensor> nd;
      auto r = attn_bwd(q, k, v, kmask, o, dO, lse, delta_in, H, D, scale, dropout_p, seed, c10::nullopt, c10::nullopt,
                        c10::nullopt, false, site, false, false, c10::nullopt, nd, {});
      dq.copy_(r[0]); dk.copy_(r[1]); dv.copy_(r[2]);
    }
    return {dq, dk, dv};
  }
  if (job.slab) pio::slab_reduce_launch(job, stream());
  Tensor dq = dq_out.has_value() ? *dq_out : torch::empty({a.B, a.Nq, H * D}, f32);
  Tensor dk = dk_out.has_value() ? *dk_out : torch::empty({a.B, a.Nk, H * D}, f32);
  Tensor dv = dv_out.has_value() ? *dv_out : torch::empty({a.B, a.Nk, H * D}, f32);
  TORCH_CHECK(dq.stride(2) == 1 && dk.stride(2) == 1 && dv.stride(2) == 1, "dq/dk/dv need unit inner stride");
  TORCH_CHECK(dq.size(0) == a.B && dq.stride(0) == a.Nq * dq.stride(1), "dq must be batch-dense");
  CHECK_DT(dq, torch::kFloat32); CHECK_DT(dk, torch::kFloat32); CHECK_DT(dv, torch::kFloat32);
  Tensor delta;
  if (delta_in.has_value()) {
    delta = *delta_in;
    TORCH_CHECK(delta.is_contiguous() && delta.numel() == (int64_t)a.B * a.Nq * H, "delta must be (B, Nq, H)");
    CHECK_DT(delta, torch::kFloat32);
  } else {
    delta = torch::empty({a.B, a.Nq, H}, f32);
  }
  const int nkb = pio::attn_bwd_key_blocks(a.Nk, (int)D);
  if (g_det && nkb > 1) {  // one dQ partial slice per key block, summed in a fixed order
    Tensor part = torch::empty({nkb, a.B, a.Nq, H * D}, f32);
    pio::attn_bwd_launch(a, (int)D, bfp(o), bfp(dO), f32p(lse), delta.data_ptr<float>(), part.data_ptr<float>(),
                         (long long)a.Nq * H * D, (int)(H * D), dk.data_ptr<float>(), dk.stride(0), (int)dk.stride(1),
                         dv.data_ptr<float>(), dv.stride(0), (int)dv.stride(1), !delta_in.has_value(), kv_accumulate,
                         (long long)a.B * a.Nq * H * D, 0, 0, stream());
    dq.narrow(2, 0, H * D).copy_(part.sum(0));
    return {dq, dk, dv};
  }
  pio::attn_bwd_launch(a, (int)D, bfp(o), bfp(dO), f32p(lse), delta.data_ptr<float>(), dq.data_ptr<float>(),
                       dq.stride(0), (int)dq.stride(1), dk.data_ptr<float>(), dk.stride(0), (int)dk.stride(1),
                       dv.data_ptr<float>(), dv.stride(0), (int)dv.stride(1), !delta_in.has_value(), kv_accumulate, 0,
                       g_det ? 0 : 1, (dq_zeroed ? 1 : 0) | (kv_zeroed ? 2 : 0), stream());
  return {dq, dk, dv};
}

// pe (optional, SURVEY K-03): x holds only the npix pixel channels of each row and row r's
// input is pe[r mod rows(pe)] — or pe[pe_index[r]] when the (R,) int64 pe_index is given (sparse
// images) — with the pixels added into its npix leading (zero) columns; pe is (M, pe_rs) fp32
// contiguous with pe_rs a multiple of 8, ≥ Kin = w.size(1)
namespace {
void pe_args(const OptT& pe, const Tensor& x, int R, int Kin, const float*& pp, int& prs, int& prows, int& npix,
             const OptT& pe_index, const long long*& pidx) {
  pp = nullptr; prs = 0; prows = 1; npix = 0; pidx = nullptr;
  TORCH_CHECK(!pe_index.has_value() || pe.has_value(), "pe_index needs a pe table");
  if (!pe.has_value()) return;
  CHECK_DT(*pe, torch::kFloat32);
  TORCH_CHECK(pe->dim() == 2 && pe->is_contiguous() && pe->size(1) % 8 == 0 && pe->size(1) >= Kin,
              "pe must be (M, pe_rs) contiguous fp32, pe_rs a multiple of 8 and >= Kin");
  if (pe_index.has_value()) {
    CHECK_DT(*pe_index, torch::kInt64);
    TORCH_CHECK(pe_index->is_contiguous() && pe_index->numel() == R, "pe_index must be R contiguous int64 rows");
    pidx = reinterpret_cast<const long long*>(pe_index->data_ptr<int64_t>());
  } else {
    TORCH_CHECK(R % pe->size(0) == 0, "rows must be a multiple of the PE rows");
  }
  TORCH_CHECK(reinterpret_cast<uintptr_t>(pe->data_ptr()) % 16 == 0, "pe must be 16-byte aligned");
  pp = pe->data_ptr<float>(); prs = (int)pe->size(1); prows = (int)pe->size(0); npix = (int)x.size(1);
  TORCH_CHECK(npix <= Kin, "more pixel channels than inputs");
}
}  // namespace

// kin (optional): the logical input width when w's rows are zero padded past it (w (N, ≥ kin))
std::vector<Tensor> ln_linear_fwd(Tensor x, OptT lnw, OptT lnb, double eps, Tensor w, OptT bias, int64_t act, OptT res,
                                  bool out_bf16, bool save_stats, OptT pe, int64_t kin, OptT pe_index) {
  CHECK_CUDA(x); CHECK_CUDA(w);
  TORCH_CHECK(x.dim() == 2 && x.stride(1) == 1, "x must be 2-D rows");
  const int R = (int)x.size(0), N = (int)w.size(0);
  const int Kin = kin >= 0 ? (int)kin : (int)w.size(1);
  TORCH_CHECK(w.dim() == 2 && w.is_contiguous() && w.size(1) >= Kin, "w must be (N, >= Kin) contiguous");
  TORCH_CHECK(pe.has_value() || x.size(1) == Kin, "x must be (R, Kin)");
  TORCH_CHECK(Kin <= 256, "Kin > 256 unsupported");
  const float* pp; int prs, prows, npix; const long long* pidx;
  pe_args(pe, x, R, Kin, pp, prs, prows, npix, pe_index, pidx);
  auto opts = x.options();
  Tensor y = torch::empty({R, N}, opts.dtype(out_bf16 ? torch::kBFloat16 : torch::kFloat32));
  Tensor mean, rstd;
  float *mp = nullptr, *rp = nullptr;
  if (save_stats && lnw.has_value()) {
    mean = torch::empty({R}, opts.dtype(torch::kFloat32));
    rstd = torch::empty({R}, opts.dtype(torch::kFloat32));
    mp = mean.data_ptr<float>(); rp = rstd.data_ptr<float>();
  }
  const float* rptr = nullptr; int res_rs = 0;
  if (res.has_value()) { rptr = f32p(*res); res_rs = (int)res->stride(0); TORCH_CHECK(res->stride(1) == 1); }
  pio::ln_linear_fwd_launch(x.data_ptr(), is_bf16(x), (int)x.stride(0), R, Kin, f32o(lnw), f32o(lnb), (float)eps, bfp(w),
                            (int)w.size(1), f32o(bias), N, (int)act, rptr, res_rs, y.data_ptr(), out_bf16, N, mp, rp, pp, prs, prows,
                            npix, pidx, stream());
  if (pidx) checked_sync("ln_linear_fwd (pe_index)");
  std::vector<Tensor> out{y};
  if (mp) { out.push_back(mean); out.push_back(rstd); }
  return out;
}

std::vector<Tensor> post_attn_fwd(Tensor o, Tensor x, Tensor wo, Tensor bo, Tensor g2, Tensor be2, double eps,
                                  Tensor w1, Tensor b1, Tensor w2, Tensor b2, OptT seed, int64_t site, double p) {
  TORCH_CHECK(o.is_contiguous() && x.is_contiguous(), "o/x must be contiguous (R, C)");
  const int R = (int)o.size(0), C = (int)o.size(1), Rx = (int)x.size(0);
  TORCH_CHECK(x.size(1) == C && Rx > 0 && R % Rx == 0, "x must be (R / k, C): row r adds x[r % rows(x)]");
  TORCH_CHECK(C == 32 || C == 64 || C == 128, "post_attn supports C in {32, 64, 128}");
  auto f32 = x.options().dtype(torch::kFloat32);
  Tensor z = torch::empty({R, C}, f32), y = torch::empty({R, C}, f32);
  Tensor m = torch::empty({R}, f32), r = torch::empty({R}, f32);
  Tensor u = torch::empty({R, C}, x.options().dtype(torch::kBFloat16));
  pio::post_attn_fwd_launch(C, bfp(o), f32p(x), bfp(wo), f32p(bo), f32p(g2), f32p(be2), (float)eps, bfp(w1), f32p(b1),
                            bfp(w2), f32p(b2), z.data_ptr<float>(), y.data_ptr<float>(), m.data_ptr<float>(),
                            r.data_ptr<float>(), bfp_mut(u), R, Rx, make_drop(seed, site, p), stream());
  return {z, y, m, r, u};
}

// self-attention layer boundary l → l+1: post-attention block of layer l, then LN1 + packed QKV
// projection of layer l+1 from the same tile.  Returns (z, y, mean2, rstd2, u, qkv, mean1, rstd1).
std::vector<Tensor> post_attn_ln_linear_fwd(Tensor o, Tensor x, Tensor wo, Tensor bo, Tensor g2, Tensor be2, double eps,
                                            Tensor w1, Tensor b1, Tensor w2, Tensor b2, Tensor lnw, Tensor lnb,
                                            Tensor wq, Tensor bq, OptT seed, int64_t site, double p) {
  TORCH_CHECK(o.is_contiguous() && x.is_contiguous(), "o/x must be contiguous (R, C)");
  const int R = (int)o.size(0), C = (int)o.size(1);
  const int Rx = (int)x.size(0);
  TORCH_CHECK(x.size(1) == C && Rx > 0 && R % Rx == 0, "x must be (R / k, C): row r adds x[r % rows(x)]");
  TORCH_CHECK(C == 32 || C == 64 || C == 128, "post_attn supports C in {32, 64, 128}");
  TORCH_CHECK(wq.is_contiguous() && wq.size(0) == 3 * C && wq.size(1) == C && bq.numel() == 3 * C,
              "wq must be the packed (3C, C) in-projection");
  TORCH_CHECK(lnw.numel() == C && lnb.numel() == C, "LN1 affine must have C entries");
  auto f32 = x.options().dtype(torch::kFloat32);
  auto b16 = x.options().dtype(torch::kBFloat16);
  Tensor z = torch::empty({R, C}, f32), y = torch::empty({R, C}, f32);
  Tensor m = torch::empty({R}, f32), r = torch::empty({R}, f32), u = torch::empty({R, C}, b16);
  Tensor qkv = torch::empty({R, 3 * C}, b16), m1 = torch::empty({R}, f32), r1 = torch::empty({R}, f32);
  pio::post_attn_ln_linear_fwd_launch(C, bfp(o), f32p(x), bfp(wo), f32p(bo), f32p(g2), f32p(be2), (float)eps, bfp(w1),
                                      f32p(b1), bfp(w2), f32p(b2), z.data_ptr<float>(), y.data_ptr<float>(),
                                      m.data_ptr<float>(), r.data_ptr<float>(), bfp_mut(u), R, Rx, f32p(lnw), f32p(lnb),
                                      bfp(wq), f32p(bq), bfp_mut(qkv), m1.data_ptr<float>(), r1.data_ptr<float>(),
                                      make_drop(seed, site, p), stream());
  return {z, y, m, r, u, qkv, m1, r1};
}

// fused latent self-attention layer forward (C = 64, H = 4, N ≤ 512 (> 256: 16-byte aligned
// operands, the chain kernel), N % 64 == 0, no attention
// dropout; residual dropout allowed): qkv (R, 3C) bf16 of this layer, x (R, C) fp32 its input →
// [o, lse, z, y, m2, r2, u] (+ [qkv, mean1, rstd1] of the next layer when lnw/lnb/wq/bq given)
std::vector<Tensor> sa_layer_fwd(Tensor qkv, Tensor x, int64_t N, double scale, Tensor wo, Tensor bo, Tensor g2,
                                 Tensor be2, double eps, Tensor w1, Tensor b1, Tensor w2, Tensor b2, OptT lnw, OptT lnb,
                                 OptT wq, OptT bq, OptT seed, int64_t site, double p) {
  const int C = 64, H = 4;
  TORCH_CHECK(qkv.is_contiguous() && x.is_contiguous(), "qkv/x must be contiguous");
  const int R = (int)x.size(0);
  TORCH_CHECK(x.size(1) == C && qkv.size(0) == R && qkv.size(1) == 3 * C, "sa_layer_fwd: C = 64, qkv (R, 192)");
  TORCH_CHECK(N > 0 && N <= 512 && N % 64 == 0 && R % N == 0, "sa_layer_fwd: N <= 512, N % 64 == 0, R = B·N");
  const bool next = wq.has_value();
  if (next)
    TORCH_CHECK(lnw.has_value() && lnb.has_value() && bq.has_value() && wq->is_contiguous() &&
                    (wq->size(0) == 3 * C || wq->size(0) == 2 * C || wq->size(0) == C) && wq->size(1) == C &&
                    bq->numel() == wq->size(0) &&
                    lnw->numel() == C && lnb->numel() == C,
                "sa_layer_fwd: next LN + projection (packed QKV (3C, C), K/V (2C, C) or a query projection (C, C))");
  const int nq = next ? (int)wq->size(0) : 3 * C;
  auto f32 = x.options().dtype(torch::kFloat32);
  auto b16 = x.options().dtype(torch::kBFloat16);
  Tensor o = torch::empty({R / N, N, C}, b16), lse = torch::empty({R / N, N, H}, f32);
  Tensor z = torch::empty({R, C}, f32), y = torch::empty({R, C}, f32);
  Tensor m = torch::empty({R}, f32), r = torch::empty({R}, f32), u = torch::empty({R, C}, b16);
  Tensor qn, m1, r1;
  if (next) { qn = torch::empty({R, nq}, b16); m1 = torch::empty({R}, f32); r1 = torch::empty({R}, f32); }
  const bool launched = pio::sa_layer_fwd_launch(bfp(qkv), (int)N, (float)(scale * 1.4426950408889634), bfp_mut(o), lse.data_ptr<float>(),
                           f32p(x), bfp(wo), f32p(bo), f32p(g2), f32p(be2), (float)eps, bfp(w1), f32p(b1), bfp(w2),
                           f32p(b2), z.data_ptr<float>(), y.data_ptr<float>(), m.data_ptr<float>(), r.data_ptr<float>(),
                           bfp_mut(u), R, next ? f32p(*lnw) : nullptr, next ? f32p(*lnb) : nullptr,
                           next ? bfp(*wq) : nullptr, next ? f32p(*bq) : nullptr, next ? bfp_mut(qn) : nullptr,
                           next ? m1.data_ptr<float>() : nullptr, next ? r1.data_ptr<float>() : nullptr,
                           make_drop(seed, site, p), nq, stream());
  TORCH_CHECK(launched, "sa_layer_fwd: every operand must be 16-byte aligned");
  if (next) return {o, lse, z, y, m, r, u, qn, m1, r1};
  return {o, lse, z, y, m, r, u};
}


// sync words of the persistent kernels (csrc/persist.hip): one zero-initialised buffer per
// (device, stream), allocated on the first launch on that stream (never during a stream capture:
// nullptr then, the caller runs the per-layer kernels), reset to zero by the last workgroup of
// every launch — launches on one stream run one after another, so they can share it
unsigned* persist_sync_buffer(const Tensor& like, int words) {
  // grown buffers are kept alive too: a captured graph may still name an older one
  static std::unordered_map<uint64_t, std::vector<Tensor>> bufs;
  hipStream_t st = stream();
  const uint64_t key = reinterpret_cast<uint64_t>(st) ^ ((uint64_t)like.get_device() << 56);
  auto& v = bufs[key];
  if (!v.empty() && v.back().numel() >= words) return reinterpret_cast<unsigned*>(v.back().data_ptr<int>());
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(st, &cs) != hipSuccess || cs != hipStreamCaptureStatusNone) return nullptr;
  // the zero fill runs on the current stream: ordered before every launch that uses the buffer
  v.push_back(torch::zeros({std::max(words, 1 << 14)}, like.options().dtype(torch::kInt32)));
  return reinterpret_cast<unsigned*>(v.back().data_ptr<int>());
}

// persistent self-attention block forward (csrc/persist.hip): every layer of a C = 64, H = 4
// block with N ≤ 256 latents in ONE launch.  Per layer i: wo..b2 (its post-attention block) and,
// for i < L - 1, the next layer's (lnw, lnb, wq, bq); the last layer optionally gets the next
// cross-attention layer's LN + query (64 rows) or K/V (128 rows) projection as an L-th entry.  Returns, per layer, [o, lse, z, y, m2, r2, u] + [qkv_n, mean_n, rstd_n] when that
// layer has a next projection.  Empty list: the operands do not qualify (the caller runs the
// per-layer kernels).
std::vector<Tensor> sa_block_fwd(Tensor qkv0, Tensor x0, int64_t N, double scale, double eps, std::vector<Tensor> wo,
                                 std::vector<Tensor> bo, std::vector<Tensor> g2, std::vector<Tensor> be2,
                                 std::vector<Tensor> w1, std::vector<Tensor> b1, std::vector<Tensor> w2,
                                 std::vector<Tensor> b2, std::vector<Tensor> lnw, std::vector<Tensor> lnb,
                                 std::vector<Tensor> wq, std::vector<Tensor> bq, OptT seed, double p) {
  const int C = 64, H = 4;
  const int L = (int)wo.size();
  TORCH_CHECK(L >= 1 && L <= pio::kPersistMaxLayers, "sa_block_fwd: 1..8 layers");
  TORCH_CHECK(bo.size() == (size_t)L && g2.size() == (size_t)L && be2.size() == (size_t)L && w1.size() == (size_t)L &&
                  b1.size() == (size_t)L && w2.size() == (size_t)L && b2.size() == (size_t)L,
              "sa_block_fwd: one post-attention parameter set per layer");
  const int nn = (int)wq.size();
  TORCH_CHECK((nn == L - 1 || nn == L) && lnw.size() == (size_t)nn && lnb.size() == (size_t)nn && bq.size() == (size_t)nn,
              "sa_block_fwd: L - 1 next projections (+ an optional last query projection)");
  TORCH_CHECK(qkv0.is_contiguous() && x0.is_contiguous(), "sa_block_fwd: contiguous qkv / x");
  const int R = (int)x0.size(0);
  TORCH_CHECK(x0.size(1) == C && qkv0.size(0) == R && qkv0.size(1) == 3 * C, "sa_block_fwd: C = 64, qkv (R, 192)");
  CHECK_DT(x0, torch::kFloat32);
  if (N <= 0 || N > 256 || N % 64 != 0 || R % N != 0 || (long long)R * 3 * C * 2 >= (1LL << 31)) return {};
  auto al = [](const void* q) { return (reinterpret_cast<uintptr_t>(q) & 15) == 0; };
  if (!al(qkv0.data_ptr()) || !al(x0.data_ptr())) return {};
  auto f32 = x0.options().dtype(torch::kFloat32);
  auto b16 = x0.options().dtype(torch::kBFloat16);
  const int B = R / (int)N;
  unsigned* sync = persist_sync_buffer(x0, pio::persist_sync_words(B));
  if (sync == nullptr) return {};
  pio::SABlockFwdArgs a{};
  a.QKV0 = bfp(qkv0);
  a.X0 = f32p(x0);
  a.sync = sync;
  a.L = L; a.N = (int)N; a.R = R;
  a.scale_log2 = (float)(scale * 1.4426950408889634);
  a.eps = (float)eps;
  a.dr = make_drop(seed, 0, p);
  std::vector<Tensor> out;
  for (int i = 0; i < L; ++i) {
    pio::SAFwdLayer& y = a.ly[i];
    for (const Tensor* t : {&wo[i], &w1[i], &w2[i]})
      TORCH_CHECK(t->is_contiguous() && t->size(0) == C && t->size(1) == C, "sa_block_fwd: (C, C) weights");
    y.Wo = bfp(wo[i]); y.W1 = bfp(w1[i]); y.W2 = bfp(w2[i]);
    y.bo = f32p(bo[i]); y.g2 = f32p(g2[i]); y.be2 = f32p(be2[i]); y.b1 = f32p(b1[i]); y.b2 = f32p(b2[i]);
    if (!al(y.Wo) || !al(y.W1) || !al(y.W2) || !al(y.g2) || !al(y.be2) || !al(y.bo) || !al(y.b1) || !al(y.b2)) return {};
    Tensor o = torch::empty({B, (int)N, C}, b16), lse = torch::empty({B, (int)N, H}, f32);
    Tensor z = torch::empty({R, C}, f32), yy = torch::empty({R, C}, f32);
    Tensor m = torch::empty({R}, f32), r = torch::empty({R}, f32), u = torch::empty({R, C}, b16);
    y.O = bfp_mut(o); y.LSE = lse.data_ptr<float>(); y.Z = z.data_ptr<float>(); y.Y = yy.data_ptr<float>();
    y.mean2 = m.data_ptr<float>(); y.rstd2 = r.data_ptr<float>(); y.U = bfp_mut(u);
    out.insert(out.end(), {o, lse, z, yy, m, r, u});
    if (i < nn) {
      const int nq = (int)wq[i].size(0);
      TORCH_CHECK(wq[i].is_contiguous() && wq[i].size(1) == C && (nq == 3 * C || (i == L - 1 && (nq == C || nq == 2 * C))) &&
                      bq[i].numel() == nq && lnw[i].numel() == C && lnb[i].numel() == C,
                  "sa_block_fwd: next projection (3C, C) (the last layer's may be a (C, C) query or (2C, C) K/V projection)");
      y.Wq = bfp(wq[i]); y.lnw = f32p(lnw[i]); y.lnb = f32p(lnb[i]); y.bq = f32p(bq[i]); y.nq = nq;
      if (!al(y.Wq) || !al(y.lnw) || !al(y.lnb) || !al(y.bq)) return {};
      Tensor qn = torch::empty({R, nq}, b16), m1 = torch::empty({R}, f32), r1 = torch::empty({R}, f32);
      y.QKVn = bfp_mut(qn); y.mean1n = m1.data_ptr<float>(); y.rstd1n = r1.data_ptr<float>();
      out.insert(out.end(), {qn, m1, r1});
    }
  }
  if (!pio::sa_block_fwd_launch(a, stream())) return {};
  return out;
}

unsigned persist_errors(bool reset) { return pio::persist_errors(reset); }

namespace {
pio::SlabJob make_job(const OptT& slab, std::vector<Tensor>& dsts, const std::vector<int64_t>& offs);
}  // namespace

// ---- per-sample latent-block kernels (csrc/sample_block.hip): C ∈ {64, 128}, H = 4, N = 32 ----
namespace {
constexpr int kSBN = 32;
void sb_check_w(const Tensor& t, int rows, int C, const char* what) {
  TORCH_CHECK(t.is_contiguous() && t.dim() == 2 && t.size(0) == rows && t.size(1) == C &&
                  t.scalar_type() == torch::kBFloat16 && (reinterpret_cast<uintptr_t>(t.data_ptr()) & 15) == 0,
              "sample block: ", what, " must be a contiguous 16-byte aligned bf16 (", rows, ", ", C, ") weight");
}
void sb_check_v(const Tensor& t, int n, const char* what) {
  TORCH_CHECK(t.is_contiguous() && t.numel() == n && t.scalar_type() == torch::kFloat32 &&
                  (reinterpret_cast<uintptr_t>(t.data_ptr()) & 15) == 0,
              "sample block: ", what, " must be a contiguous 16-byte aligned fp32 vector of ", n);
}
// per layer the 12 parameters in layer_spec_and_params order with the bf16 weight shadows:
// (g1, be1, wqkv_bf16, bqkv, wo_bf16, bo, g2, be2, w1_bf16, b1, w2_bf16, b2)
void sb_fill_params(pio::SBLayer& y, const std::vector<Tensor>& p, int i, int C) {
  const Tensor* q = &p[12 * i];
  sb_check_v(q[0], C, "γ1"); sb_check_v(q[1], C, "β1"); sb_check_w(q[2], 3 * C, C, "Wqkv");
  sb_check_v(q[3], 3 * C, "bqkv"); sb_check_w(q[4], C, C, "Wo"); sb_check_v(q[5], C, "bo");
  sb_check_v(q[6], C, "γ2"); sb_check_v(q[7], C, "β2"); sb_check_w(q[8], C, C, "W1");
  sb_check_v(q[9], C, "b1"); sb_check_w(q[10], C, C, "W2"); sb_check_v(q[11], C, "b2");
  y.g1 = f32p(q[0]); y.be1 = f32p(q[1]); y.Wqkv = bfp(q[2]); y.bqkv = f32p(q[3]); y.Wo = bfp(q[4]); y.bo = f32p(q[5]);
  y.g2 = f32p(q[6]); y.be2 = f32p(q[7]); y.W1 = bfp(q[8]); y.b1 = f32p(q[9]); y.W2 = bfp(q[10]); y.b2 = f32p(q[11]);
}
constexpr int kSBSaved = 12;  // LN1X QKV O LN2Y U GU Y Z mean1 rstd1 mean2 rstd2
void sb_fill_saved(pio::SBLayer& y, const std::vector<Tensor>& sv, int i, int R, int C) {
  const Tensor* t = &sv[kSBSaved * i];
  for (int k = 0; k < kSBSaved; ++k) {
    const int64_t want = k < 8 ? (int64_t)R * (k == 1 ? 3 * C : C) : R;
    TORCH_CHECK(t[k].is_contiguous() && t[k].numel() == want &&
                    t[k].scalar_type() == (k < 6 ? torch::kBFloat16 : torch::kFloat32),
                "sample block: saved tensor ", k, " of layer ", i, " has the wrong shape / dtype");
  }
  y.LN1X = reinterpret_cast<uint16_t*>(t[0].data_ptr()); y.QKV = reinterpret_cast<uint16_t*>(t[1].data_ptr());
  y.O = reinterpret_cast<uint16_t*>(t[2].data_ptr()); y.LN2Y = reinterpret_cast<uint16_t*>(t[3].data_ptr());
  y.U = reinterpret_cast<uint16_t*>(t[4].data_ptr()); y.GU = reinterpret_cast<uint16_t*>(t[5].data_ptr());
  y.Y = t[6].data_ptr<float>(); y.Z = t[7].data_ptr<float>(); y.mean1 = t[8].data_ptr<float>();
  y.rstd1 = t[9].data_ptr<float>(); y.mean2 = t[10].data_ptr<float>(); y.rstd2 = t[11].data_ptr<float>();
}
}  // namespace

// the pre stage's 10 tensors: [O (R, C) bf16, x_q (R, C) or (32, C) fp32, wo_bf16, bo, g2, be2,
// w1_bf16, b1, w2_bf16, b2]
namespace {
void sb_fill_pre(pio::SBLayer& y, const std::vector<Tensor>& pre, int C) {
  sb_check_w(pre[2], C, C, "pre Wo"); sb_check_v(pre[3], C, "pre bo"); sb_check_v(pre[4], C, "pre γ2");
  sb_check_v(pre[5], C, "pre β2"); sb_check_w(pre[6], C, C, "pre W1"); sb_check_v(pre[7], C, "pre b1");
  sb_check_w(pre[8], C, C, "pre W2"); sb_check_v(pre[9], C, "pre b2");
  y.Wo = bfp(pre[2]); y.bo = f32p(pre[3]); y.g2 = f32p(pre[4]); y.be2 = f32p(pre[5]);
  y.W1 = bfp(pre[6]); y.b1 = f32p(pre[7]); y.W2 = bfp(pre[8]); y.b2 = f32p(pre[9]);
}
constexpr int kSBPreSaved = 6;  // LN2Y U GU (bf16) Y mean2 rstd2 (fp32)
void sb_fill_pre_saved(pio::SBLayer& y, const std::vector<Tensor>& sv, int R, int C) {
  TORCH_CHECK((int)sv.size() == kSBPreSaved, "sample block: 6 saved pre-stage tensors");
  for (int k = 0; k < kSBPreSaved; ++k) {
    const int64_t want = k < 4 ? (int64_t)R * C : R;
    TORCH_CHECK(sv[k].is_contiguous() && sv[k].numel() == want &&
                    sv[k].scalar_type() == (k < 3 ? torch::kBFloat16 : torch::kFloat32),
                "sample block: saved pre-stage tensor ", k, " has the wrong shape / dtype");
  }
  y.LN2Y = reinterpret_cast<uint16_t*>(sv[0].data_ptr()); y.U = reinterpret_cast<uint16_t*>(sv[1].data_ptr());
  y.GU = reinterpret_cast<uint16_t*>(sv[2].data_ptr()); y.Y = sv[3].data_ptr<float>();
  y.mean2 = sv[4].data_ptr<float>(); y.rstd2 = sv[5].data_ptr<float>();
}
void sb_check_pre_o(const Tensor& o, int R, int C) {
  TORCH_CHECK(o.is_contiguous() && o.dim() == 2 && o.size(0) == R && o.size(1) == C && o.scalar_type() == torch::kBFloat16 &&
                  (reinterpret_cast<uintptr_t>(o.data_ptr()) & 15) == 0,
              "sample block: pre O must be (B·32, C) contiguous bf16");
}
}  // namespace

// forward of a whole block, one workgroup per sample: x (B·32, C) fp32 → per layer
// [LN1X, QKV, O, LN2Y, U, GU (bf16), Y, Z, mean1, rstd1, mean2, rstd2 (fp32)]; the block output is
// the last layer's Z.  pre (10 tensors, see sb_fill_pre): the cross layer's post-attention half
// runs first and WRITES x (its output, the block input); its 6 saved tensors are appended.
// post (4 tensors [γq, βq, wq_bf16 (C, C), bq]): the next cross layer's LN + query projection of the
// block output; [Q (R, C) bf16, LN_q(z) (R, C) bf16, mean, rstd] are appended (after pre's)
namespace {
void sb_fill_post(pio::SBQPath& q, const std::vector<Tensor>& post, int C) {
  TORCH_CHECK(post.size() == 4, "sample block: post = [γ, β, w (N, C) bf16, bias (N)], N ∈ {C, 2C}");
  const int N = post[2].dim() == 2 ? (int)post[2].size(0) : 0;
  TORCH_CHECK(N == C || N == 2 * C, "sample block: the post projection has C or 2C outputs");
  sb_check_v(post[0], C, "post γ"); sb_check_v(post[1], C, "post β"); sb_check_w(post[2], N, C, "post W");
  sb_check_v(post[3], N, "post bias");
  q.N = N; q.g = f32p(post[0]); q.b = f32p(post[1]); q.Wq = bfp(post[2]); q.bq = f32p(post[3]);
}
}  // namespace

std::vector<Tensor> sb_fwd(Tensor x, std::vector<Tensor> params, double scale, double eps, std::vector<Tensor> pre,
                           std::vector<Tensor> post) {
  const int C = x.dim() == 2 ? (int)x.size(1) : 0;
  TORCH_CHECK(x.is_contiguous() && (C == 64 || C == 128) && x.size(0) % kSBN == 0 && x.size(0) > 0,
              "sb_fwd: x (B·32, C), C ∈ {64, 128}");
  CHECK_DT(x, torch::kFloat32);
  const int L = (int)params.size() / 12, R = (int)x.size(0);
  TORCH_CHECK(L >= 1 && L <= pio::kSBMaxLayers && (int)params.size() == 12 * L, "sb_fwd: 1..4 layers × 12 parameters");
  auto f32 = x.options().dtype(torch::kFloat32);
  auto b16 = x.options().dtype(torch::kBFloat16);
  pio::SBFwdArgs a{};
  a.X0 = f32p(x); a.L = L; a.B = R / kSBN;
  a.scale_log2 = (float)(scale * 1.4426950408889634);
  a.eps = (float)eps;
  std::vector<Tensor> out;
  for (int i = 0; i < L; ++i) {
    sb_fill_params(a.ly[i], params, i, C);
    std::vector<Tensor> sv{torch::empty({R, C}, b16), torch::empty({R, 3 * C}, b16), torch::empty({R, C}, b16),
                           torch::empty({R, C}, b16), torch::empty({R, C}, b16), torch::empty({R, C}, b16),
                           torch::empty({R, C}, f32), torch::empty({R, C}, f32), torch::empty({R}, f32),
                           torch::empty({R}, f32), torch::empty({R}, f32), torch::empty({R}, f32)};
    out.insert(out.end(), sv.begin(), sv.end());
    sb_fill_saved(a.ly[i], out, i, R, C);
  }
  if (!pre.empty()) {
    TORCH_CHECK(pre.size() == 10, "sb_fwd: pre = [O, x_q, wo, bo, g2, be2, w1, b1, w2, b2]");
    sb_check_pre_o(pre[0], R, C);
    const Tensor& xq = pre[1];
    TORCH_CHECK(xq.is_contiguous() && xq.dim() == 2 && xq.size(1) == C && (xq.size(0) == R || xq.size(0) == kSBN) &&
                    xq.scalar_type() == torch::kFloat32,
                "sb_fwd: pre x_q must be (B·32, C) or broadcast (32, C) fp32");
    sb_fill_pre(a.pre, pre, C);
    std::vector<Tensor> sv{torch::empty({R, C}, b16), torch::empty({R, C}, b16), torch::empty({R, C}, b16),
                           torch::empty({R, C}, f32), torch::empty({R}, f32), torch::empty({R}, f32)};
    sb_fill_pre_saved(a.pre, sv, R, C);
    a.pre.Z = x.data_ptr<float>();
    a.preO = bfp(pre[0]);
    a.preX = f32p(xq);
    a.preX_bs = xq.size(0) == R ? kSBN : 0;
    a.has_pre = 1;
    out.insert(out.end(), sv.begin(), sv.end());
  }
  if (!post.empty()) {
    sb_fill_post(a.post, post, C);
    Tensor q = torch::empty({R, (int64_t)a.post.N}, b16), lnx = torch::empty({R, C}, b16), mean = torch::empty({R}, f32),
           rstd = torch::empty({R}, f32);
    a.post.Q = reinterpret_cast<uint16_t*>(q.data_ptr()); a.post.LNX = reinterpret_cast<uint16_t*>(lnx.data_ptr());
    a.post.mean = mean.data_ptr<float>(); a.post.rstd = rstd.data_ptr<float>();
    a.has_post = 1;
    out.insert(out.end(), {q, lnx, mean, rstd});
  }
  TORCH_CHECK(pio::sb_fwd_launch(a, C, stream()), "sb_fwd: launch refused");
  return out;
}

// backward of a block: dz (B·32, C) fp32, x0 the block input, saved = sb_fwd's outputs, params
// as sb_fwd's.  Returns [dx, the (B, 4·L·C) fp32 LayerNorm partial slab (row b: sample b's
// [dγ1 | dβ1 | dγ2 | dβ2] of layer 0, then layer 1, …; sum the rows into the gradients), then per
// layer the gradient rows dQKV, dY, dU, dZ (bf16)] for sb_wgrad
// pre (as sb_fwd's, x_q unused) + pre_saved (sb_fwd's 6 appended tensors): the cross layer's
// post-attention backward runs last; dx is then the gradient of its residual input x_q, and
// [dO (R, C) bf16, δ (R, 4) fp32, dY, dU, dZ (bf16 rows)] are appended; the LayerNorm slab rows
// are 2C wider (the pre stage's dγ2 | dβ2 last).  zero_out: an fp32 buffer of 4k elements the
// kernel clears (the cross attention backward's accumulators)
// post (as sb_fwd's) + post_io [dQ (R, C) fp32, dres (R, C) fp32, mean, rstd (sb_fwd's)]: the query
// path's backward runs first, dz is then unused; [dQ bf16 rows] is appended, the slab rows 2C wider
std::vector<Tensor> sb_bwd(Tensor dz, Tensor x0, std::vector<Tensor> saved, std::vector<Tensor> params, double scale,
                           double eps, std::vector<Tensor> pre, std::vector<Tensor> pre_saved, OptT zero_out,
                           std::vector<Tensor> post, std::vector<Tensor> post_io) {
  const int C = x0.dim() == 2 ? (int)x0.size(1) : 0;
  TORCH_CHECK(dz.is_contiguous() && x0.is_contiguous() && dz.sizes() == x0.sizes() && (C == 64 || C == 128) &&
                  x0.size(0) % kSBN == 0 && x0.size(0) > 0,
              "sb_bwd: dz / x0 (B·32, C), C ∈ {64, 128}");
  CHECK_DT(dz, torch::kFloat32);
  CHECK_DT(x0, torch::kFloat32);
  const int L = (int)params.size() / 12, R = (int)x0.size(0);
  TORCH_CHECK(L >= 1 && L <= pio::kSBMaxLayers && (int)params.size() == 12 * L && (int)saved.size() == kSBSaved * L,
              "sb_bwd: saved per layer");
  auto f32 = x0.options().dtype(torch::kFloat32);
  auto b16 = x0.options().dtype(torch::kBFloat16);
  pio::SBBwdArgs a{};
  a.X0 = f32p(x0); a.dZ = f32p(dz); a.L = L; a.B = R / kSBN;
  a.scale_log2 = (float)(scale * 1.4426950408889634);
  a.eps = (float)eps;
  Tensor dx = torch::empty({R, C}, f32);
  a.dX = dx.data_ptr<float>();
  const bool hp = !pre.empty(), hq = !post.empty();
  a.ln_rs = 4 * L * C + (hp ? 2 * C : 0) + (hq ? 2 * C : 0);
  Tensor lns = torch::empty({(int64_t)a.B, (int64_t)a.ln_rs}, f32);  // every element stored by the kernel
  std::vector<Tensor> out{dx, lns};
  for (int i = 0; i < L; ++i) {
    sb_fill_params(a.ly[i], params, i, C);
    sb_fill_saved(a.ly[i], saved, i, R, C);
    pio::SBGrad& g = a.gr[i];
    Tensor dq = torch::empty({R, 3 * C}, b16), dy = torch::empty({R, C}, b16), du = torch::empty({R, C}, b16),
           dzz = torch::empty({R, C}, b16);
    g.dQKV = reinterpret_cast<uint16_t*>(dq.data_ptr()); g.dY = reinterpret_cast<uint16_t*>(dy.data_ptr());
    g.dU = reinterpret_cast<uint16_t*>(du.data_ptr()); g.dZ = reinterpret_cast<uint16_t*>(dzz.data_ptr());
    float* lp = lns.data_ptr<float>() + (int64_t)4 * i * C;
    g.dg1 = lp; g.dbe1 = lp + C; g.dg2 = lp + 2 * C; g.dbe2 = lp + 3 * C;
    out.insert(out.end(), {dq, dy, du, dzz});
  }
  if (hp) {
    TORCH_CHECK(pre.size() == 10, "sb_bwd: pre = [O, x_q, wo, bo, g2, be2, w1, b1, w2, b2]");
    sb_check_pre_o(pre[0], R, C);
    sb_fill_pre(a.pre, pre, C);
    sb_fill_pre_saved(a.pre, pre_saved, R, C);
    a.pre.O = reinterpret_cast<uint16_t*>(pre[0].data_ptr());
    Tensor dO = torch::empty({R, C}, b16), delta = torch::empty({R, 4}, f32), dy = torch::empty({R, C}, b16),
           du = torch::empty({R, C}, b16), dzz = torch::empty({R, C}, b16);
    a.preDO = reinterpret_cast<uint16_t*>(dO.data_ptr());
    a.preDelta = delta.data_ptr<float>();
    pio::SBGrad& g = a.pgr;
    g.dY = reinterpret_cast<uint16_t*>(dy.data_ptr()); g.dU = reinterpret_cast<uint16_t*>(du.data_ptr());
    g.dZ = reinterpret_cast<uint16_t*>(dzz.data_ptr());
    float* lp = lns.data_ptr<float>() + (int64_t)4 * L * C;
    g.dg2 = lp; g.dbe2 = lp + C;
    a.has_pre = 1;
    out.insert(out.end(), {dO, delta, dy, du, dzz});
  }
  if (hq) {
    sb_fill_post(a.post, post, C);
    TORCH_CHECK(post_io.size() == 4, "sb_bwd: post_io = [dQ, dres (or empty), mean, rstd]");
    const bool has_dres = post_io[1].numel() > 0;
    for (int k = 0; k < 4; ++k) {
      if (k == 1 && !has_dres) continue;
      const int64_t want = k == 0 ? (int64_t)R * a.post.N : (k == 1 ? (int64_t)R * C : R);
      CHECK_DT(post_io[k], torch::kFloat32);
      TORCH_CHECK(post_io[k].is_contiguous() && post_io[k].numel() == want &&
                      (reinterpret_cast<uintptr_t>(post_io[k].data_ptr()) & 15) == 0,
                  "sb_bwd: post_io tensor ", k, " must be contiguous fp32 (R, N) / (R, C) / (R)");
    }
    a.post.dQ = f32p(post_io[0]); a.post.dres = has_dres ? f32p(post_io[1]) : nullptr;
    a.post.mean = post_io[2].data_ptr<float>(); a.post.rstd = post_io[3].data_ptr<float>();
    Tensor dqb = torch::empty({R, (int64_t)a.post.N}, b16);
    a.post.dQb = reinterpret_cast<uint16_t*>(dqb.data_ptr());
    float* lp = lns.data_ptr<float>() + (int64_t)(4 * L + (hp ? 2 : 0)) * C;
    a.post.dg = lp; a.post.db = lp + C;
    a.has_post = 1;
    out.push_back(dqb);
  }
  if (zero_out.has_value()) {
    CHECK_DT(*zero_out, torch::kFloat32);
    TORCH_CHECK(zero_out->is_contiguous() && zero_out->numel() % 4 == 0 &&
                    reinterpret_cast<uintptr_t>(zero_out->data_ptr()) % 16 == 0,
                "sb_bwd: zero_out must be a contiguous, 16-byte aligned fp32 buffer of 4k elements");
    a.zero_p = zero_out->data_ptr<float>();
    a.zero_n4 = zero_out->numel() / 4;
  }
  TORCH_CHECK(pio::sb_bwd_launch(a, C, stream()), "sb_bwd: launch refused");
  return out;
}

// grouped weight gradients of a block: jobs = [G (R, N) bf16, A (R, C) bf16, dW (N, C) fp32,
// db (N) fp32] × n (added to dW / db); one C for every job.  job_slab / job_dsts / job_offs: a
// slab reduction run by appended workgroups (the block's LayerNorm partials from sb_bwd)
void sb_wgrad(std::vector<Tensor> jobs, OptT job_slab, std::vector<Tensor> job_dsts, std::vector<int64_t> job_offs) {
  TORCH_CHECK(jobs.size() % 4 == 0 && !jobs.empty() && (int)jobs.size() / 4 <= pio::kSBMaxJobs, "sb_wgrad: 1..", pio::kSBMaxJobs, " jobs");
  pio::SBWgradArgs a{};
  a.njobs = (int)jobs.size() / 4;
  a.R = (int)jobs[0].size(0);
  const int C = jobs[1].dim() == 2 ? (int)jobs[1].size(1) : 0;
  TORCH_CHECK(C == 64 || C == 128, "sb_wgrad: A (R, C), C ∈ {64, 128}");
  for (int j = 0; j < a.njobs; ++j) {
    const Tensor &G = jobs[4 * j], &A = jobs[4 * j + 1], &dW = jobs[4 * j + 2], &db = jobs[4 * j + 3];
    const int N = (int)G.size(1);
    TORCH_CHECK(G.is_contiguous() && A.is_contiguous() && G.dim() == 2 && A.dim() == 2 && G.size(0) == a.R &&
                    A.size(0) == a.R && A.size(1) == C && G.scalar_type() == torch::kBFloat16 &&
                    A.scalar_type() == torch::kBFloat16 && N % 64 == 0 && N > 0,
                "sb_wgrad: G (R, N) / A (R, C) bf16");
    TORCH_CHECK(dW.is_contiguous() && dW.numel() == (int64_t)N * C && db.is_contiguous() && db.numel() == N,
                "sb_wgrad: dW (N, C) / db (N)");
    CHECK_DT(dW, torch::kFloat32);
    CHECK_DT(db, torch::kFloat32);
    a.job[j] = pio::SBWgradJob{bfp(G), bfp(A), dW.data_ptr<float>(), db.data_ptr<float>(), N, 0};
  }
  TORCH_CHECK(pio::sb_wgrad_launch(a, C, make_job(job_slab, job_dsts, job_offs), stream()), "sb_wgrad: launch refused");
}

// workgroups of a non-deterministic SlabJob (128 measured best on the MLM step: 96–128 ≈ equal,
// 192 and 256 slower: profiles/r5_ab/README.md)
int slab_job_target() { return 128; }

// the backward entry points below ACCUMULATE parameter gradients into caller-provided fp32
// tensors (normally views of the flat gradient buffer) with device atomics: no partial slabs,
// no reduction pass, no autograd AccumulateGrad adds
namespace {
float* grad_target(Tensor& t, int64_t numel, const char* what) {
  TORCH_CHECK(t.is_contiguous() && t.numel() == numel, "bad gradient target ", what);
  CHECK_DT(t, torch::kFloat32);
  return t.data_ptr<float>();
}
constexpr int kGradReplicas = 8;
// gradient target: K contiguous floats (any shape), or an (8, K) replica view with unit inner
// stride whose row stride is shared by every target of the call (workgroup i adds into row
// i % 8).  A 2-D target counts as replicated only when it is (8, K) with K == its numel / 8.
// Slab mode (slab_rows > 0): every target is an (slab_rows, K) view of ONE (tiles, P) slab —
// workgroup i stores its partial into row i (no atomics; ops/fused.py reduces the slab).
float* vec_target(Tensor& t, int64_t K, const char* what, int& vrs, int64_t slab_rows = 0) {
  CHECK_DT(t, torch::kFloat32);
  if (slab_rows > 0) {
    TORCH_CHECK(t.dim() == 2 && t.size(0) == slab_rows && t.size(1) == K && t.stride(1) == 1,
                "slab target ", what, " must be a (tiles, K) view");
    TORCH_CHECK(vrs < 0 || vrs == (int)t.stride(0), "slab targets must share one row stride");
    vrs = (int)t.stride(0);
  } else if (t.dim() == 2 && t.size(0) == kGradReplicas && t.size(1) == K) {
    TORCH_CHECK(t.stride(1) == 1, "bad replicated target ", what);
    TORCH_CHECK(vrs < 0 || vrs == (int)t.stride(0), "replicated targets must share one row stride");
    vrs = (int)t.stride(0);
  } else {
    TORCH_CHECK(t.is_contiguous() && t.numel() == K, "bad gradient target ", what);
    TORCH_CHECK(vrs <= 0, "mixing replicated and plain vector targets");
    vrs = 0;
  }
  return t.data_ptr<float>();
}
// a slab reduction job: dsts[j] += Σ_rows slab[:, offs[j] : offs[j] + dsts[j].numel()]
// (slab (S, P) contiguous fp32, P and every offset multiples of 4, ≤ 8 segments)
pio::SlabJob make_job(const OptT& slab, std::vector<Tensor>& dsts, const std::vector<int64_t>& offs) {
  pio::SlabJob j{};
  if (!slab.has_value()) return j;
  const Tensor& t = *slab;
  CHECK_DT(t, torch::kFloat32);
  TORCH_CHECK(t.dim() == 2 && t.is_contiguous() && t.size(1) % 4 == 0, "slab must be (S, P), P % 4 == 0");
  TORCH_CHECK(dsts.size() == offs.size() && dsts.size() <= (size_t)pio::kMaxSlabSegs, "slab job: ≤ 16 segments");
  const int P = (int)t.size(1);
  for (size_t q = 0; q < dsts.size(); ++q) {
    Tensor& d = dsts[q];
    CHECK_DT(d, torch::kFloat32);
    TORCH_CHECK(d.is_contiguous() && d.device() == t.device(), "slab job: destinations must be contiguous");
    TORCH_CHECK(offs[q] % 4 == 0 && offs[q] >= 0 && offs[q] + d.numel() <= P, "slab job: bad segment");
    if (d.numel() == 0) continue;
    j.dst[j.n] = d.data_ptr<float>(); j.off[j.n] = (int)offs[q]; j.len[j.n] = (int)d.numel(); ++j.n;
  }
  if (j.n == 0 || t.size(0) == 0) return j;
  j.slab = t.data_ptr<float>();
  j.S = (int)t.size(0);
  j.P = P;
  j.det = g_det ? 1 : 0;
  if (g_det) {  // one workgroup per 256 columns, all rows (common.h slab_reduce_block)
    j.nbx = (P + 255) / 256;
    j.nblk = j.nbx;
  } else {  // 1024-column blocks × row splits: ≈ slab_job_target() workgroups, one round
    j.nbx = (P + pio::kSlabColsPerBlock - 1) / pio::kSlabColsPerBlock;
    int nsy = std::max(1, std::min(j.S, slab_job_target() / j.nbx));
    const int rb = (j.S + nsy - 1) / nsy;
    nsy = (j.S + rb - 1) / rb;
    j.nblk = j.nbx * nsy;
  }
  return j;
}

// zero_out (optional): an fp32 buffer the kernel carrying this job clears on the way (the NEXT
// kernel's atomic accumulator, e.g. the cross-attention dQ) — no separate fill launch
pio::SlabJob with_zero_span(pio::SlabJob job, const OptT& zero_out, const Tensor& like) {
  if (zero_out.has_value()) {
    CHECK_DT(*zero_out, torch::kFloat32);
    TORCH_CHECK(zero_out->is_contiguous() && zero_out->numel() % 4 == 0 && zero_out->get_device() == like.get_device() &&
                    reinterpret_cast<uintptr_t>(zero_out->data_ptr()) % 16 == 0,
                "zero_out must be a contiguous, 16-byte aligned fp32 buffer of 4k elements");
    job.zero_p = zero_out->data_ptr<float>();
    job.zero_n4 = zero_out->numel() / 4;
  }
  return job;
}
}  // namespace

// grads = [dWo, dbo, dg2, dbe2, dW1, db1, dW2, db2]; returns (dy, dO, delta)
// slab: targets are (ceil(R/64), ·) views of one slab (see vec_target), reduced by slab_reduce
std::vector<Tensor> post_attn_bwd(Tensor dz, Tensor y, Tensor m2, Tensor r2, Tensor u, Tensor o, Tensor wo, Tensor w1,
                                  Tensor w2, Tensor g2, Tensor be2, int64_t H, std::vector<Tensor> grads, bool slab,
                                  OptT job_slab, std::vector<Tensor> job_dsts, std::vector<int64_t> job_offs,
                                  OptT seed, int64_t site, double p, OptT zero_out) {
  TORCH_CHECK(dz.is_contiguous() && y.is_contiguous() && u.is_contiguous() && o.is_contiguous(),
              "post_attn_bwd operands must be contiguous (R, C)");
  const int R = (int)dz.size(0), C = (int)dz.size(1);
  TORCH_CHECK(C == 32 || C == 64 || C == 128, "post_attn supports C in {32, 64, 128}");
  TORCH_CHECK(H > 0 && C % H == 0, "heads must divide C");
  TORCH_CHECK(grads.size() == 8, "post_attn_bwd needs 8 gradient targets");
  TORCH_CHECK(!g_det || slab, "deterministic mode: post_attn_bwd parameter gradients need slab mode (R < 2^17 rows)");
  const int64_t CC = (int64_t)C * C;
  int vrs = -1;
  const int64_t sr = slab ? (R + 63) / 64 : 0;
  pio::PostAttnGrads pg{vec_target(grads[0], CC, "dWo", vrs, sr), vec_target(grads[1], C, "dbo", vrs, sr),
                        vec_target(grads[2], C, "dg2", vrs, sr), vec_target(grads[3], C, "dbe2", vrs, sr),
                        vec_target(grads[4], CC, "dW1", vrs, sr), vec_target(grads[5], C, "db1", vrs, sr),
                        vec_target(grads[6], CC, "dW2", vrs, sr), vec_target(grads[7], C, "db2", vrs, sr), 0, 0};
  pg.vrs = vrs < 0 ? 0 : vrs;
  pg.slab = slab ? 1 : 0;
  auto f32 = dz.options().dtype(torch::kFloat32);
  Tensor dy = torch::empty({R, C}, f32);
  Tensor dO = torch::empty({R, C}, dz.options().dtype(torch::kBFloat16));
  Tensor delta = torch::empty({R, H}, f32);
  pio::SlabJob job = with_zero_span(make_job(job_slab, job_dsts, job_offs), zero_out, dz);
  pio::post_attn_bwd_launch(C, f32p(dz), f32p(y), f32p(m2), f32p(r2), bfp(u), bfp(o), bfp(wo), bfp(w1), bfp(w2),
                            f32p(g2), f32p(be2), dy.data_ptr<float>(), bfp_mut(dO), delta.data_ptr<float>(), (int)H,
                            pg, R, job, make_drop(seed, site, p), stream());
  return {dy, dO, delta};
}

// self-attention layer boundary l+1 → l, backward, slab mode only: the LN1+QKV backward of
// layer l+1 (g = dQKV (R, 3C) fp32, dres = dY_{l+1}) produces dZ_l in registers, the
// post-attention backward of layer l consumes it.  ll_grads = slab views for (dγ1, dβ1, dWqkv,
// dbqkv) of layer l+1, pa_grads = the 8 post-attention slab views of layer l — all of ONE slab.
// Returns (dy, dO, delta) of layer l.
std::vector<Tensor> ln_linear_post_attn_bwd(Tensor g, Tensor wq, Tensor x, Tensor mean1, Tensor rstd1, Tensor lnw,
                                            Tensor lnb, Tensor dres, std::vector<Tensor> ll_grads, Tensor y, Tensor m2,
                                            Tensor r2, Tensor u, Tensor o, Tensor wo, Tensor w1, Tensor w2, Tensor g2,
                                            Tensor be2, int64_t H, std::vector<Tensor> pa_grads, OptT job_slab,
                                            std::vector<Tensor> job_dsts, std::vector<int64_t> job_offs, OptT seed,
                                            int64_t site, double p, OptT zero_out, OptT att_qkv, OptT att_lse,
                                            OptT att_out, double att_scale) {
  TORCH_CHECK(y.is_contiguous() && u.is_contiguous() && o.is_contiguous() && x.is_contiguous() && dres.is_contiguous(),
              "operands must be contiguous (R, C)");
  const int R = (int)y.size(0), C = (int)y.size(1);
  TORCH_CHECK(C == 32 || C == 64 || C == 128, "the fused self-attention backward supports C in {32, 64, 128}");
  TORCH_CHECK(H > 0 && C % H == 0, "heads must divide C");
  const int nq = (int)wq.size(0);  // 3C: packed QKV of a self-attention layer; C: a cross-attention query projection
  TORCH_CHECK(wq.is_contiguous() && (nq == 3 * C || nq == C) && wq.size(1) == C, "wq must be (3C, C) or (C, C)");
  TORCH_CHECK(g.is_contiguous() && g.size(0) == R && g.size(1) == nq, "g must be (R, rows(wq)) contiguous");
  TORCH_CHECK(g.scalar_type() == torch::kFloat32 || g.scalar_type() == torch::kBFloat16, "g must be fp32 or bf16");
  TORCH_CHECK(x.size(0) == R && x.size(1) == C && dres.size(0) == R && dres.size(1) == C, "x / dres must be (R, C)");
  TORCH_CHECK(ll_grads.size() == 4 && pa_grads.size() == 8, "4 + 8 slab targets expected");
  const int64_t sr = (R + 63) / 64, CC = (int64_t)C * C;
  int vrs = -1;
  auto T = [&](Tensor& t, int64_t K, const char* what) { return vec_target(t, K, what, vrs, sr); };
  float* dg1 = T(ll_grads[0], C, "dlnw");
  float* db1 = T(ll_grads[1], C, "dlnb");
  float* dwq = T(ll_grads[2], (int64_t)nq * C, "dWqkv");
  float* dbq = T(ll_grads[3], nq, "dbqkv");
  pio::PostAttnGrads pg{T(pa_grads[0], CC, "dWo"), T(pa_grads[1], C, "dbo"), T(pa_grads[2], C, "dg2"),
                        T(pa_grads[3], C, "dbe2"), T(pa_grads[4], CC, "dW1"), T(pa_grads[5], C, "db1"),
                        T(pa_grads[6], CC, "dW2"), T(pa_grads[7], C, "db2"), vrs, 1};
  auto f32 = y.options().dtype(torch::kFloat32);
  Tensor dy = torch::empty({R, C}, f32);
  Tensor dO = torch::empty({R, C}, y.options().dtype(torch::kBFloat16));
  Tensor delta = torch::empty({R, H}, f32);
  const auto job = with_zero_span(make_job(job_slab, job_dsts, job_offs), zero_out, y);
  const auto dr = make_drop(seed, site, p);
  // att_*: the layer below's attention backward fused in (N = 64 latents per sample, the tile is
  // the sample): its packed QKV rows and LSE in, its dQKV (R, 3C) bf16 out; dO / delta are then
  // not produced (the returned tensors are unwritten)
  const uint16_t* aq = nullptr; const float* al = nullptr; uint16_t* ao = nullptr;
  if (att_out.has_value()) {
    TORCH_CHECK(att_qkv.has_value() && att_lse.has_value(), "att_out needs att_qkv and att_lse");
    CHECK_DT(*att_qkv, torch::kBFloat16); CHECK_DT(*att_out, torch::kBFloat16); CHECK_DT(*att_lse, torch::kFloat32);
    TORCH_CHECK(C == 64 && H == 4 && R % 64 == 0, "fused attention backward: C = 64, H = 4, R % 64 == 0");
    TORCH_CHECK(att_qkv->is_contiguous() && att_qkv->numel() == (int64_t)R * 3 * C && att_out->is_contiguous() &&
                    att_out->numel() == (int64_t)R * 3 * C && att_lse->is_contiguous() && att_lse->numel() == (int64_t)R * H,
                "fused attention backward: qkv / out (R, 3C), lse (R, H) contiguous");
    aq = bfp(*att_qkv); al = f32p(*att_lse); ao = bfp_mut(*att_out);
  }
  auto launch = [&](const Tensor& gg) {
    const bool gbf = gg.scalar_type() == torch::kBFloat16;
    return pio::ln_linear_post_attn_bwd_launch(
        C, gg.data_ptr(), gbf, bfp(wq), f32p(x), f32p(mean1), f32p(rstd1), f32p(lnw), f32p(lnb), f32p(dres), dg1, db1,
        dwq, dbq, f32p(y), f32p(m2), f32p(r2), bfp(u), bfp(o), bfp(wo), bfp(w1), bfp(w2), f32p(g2), f32p(be2),
        dy.data_ptr<float>(), bfp_mut(dO), delta.data_ptr<float>(), (int)H, pg, R, job, dr, nq, aq, al, ao,
        (float)att_scale, stream());
  };
  // a bf16 G (from attn_bwd's bf16 outputs) is taken by the chain-layout kernel; any other
  // kernel gets it widened to fp32 (same values)
  if (!launch(g)) TORCH_CHECK(!ao && launch(g.to(torch::kFloat32)), "ln_linear_post_attn_bwd: launch failed");
  return {dy, dO, delta};
}

// dX = LN_bwd(g·w) (+ dres); accumulates dγ/dβ (dlnw/dlnb, needed when lnw is given) and, when
// dW is given, dW += gᵀ·LN(x) and db += Σ_rows g.  Returns dX when need_dx.
constexpr int kTallRows = 1 << 17;

OptT ln_linear_bwd(Tensor g, Tensor w, Tensor x, OptT mean, OptT rstd, OptT lnw, OptT lnb, OptT dres, bool need_dx,
                   OptT dlnw, OptT dlnb, OptT dW, OptT db, OptT pe, int64_t kin, bool slab, OptT job_slab,
                   std::vector<Tensor> job_dsts, std::vector<int64_t> job_offs, OptT dx_out, OptT pe_index) {
  TORCH_CHECK(g.dim() == 2 && g.stride(1) == 1 && x.dim() == 2 && x.stride(1) == 1, "g / x must be 2-D rows");
  const int R = (int)g.size(0), N = (int)g.size(1);
  TORCH_CHECK(!(slab && R >= kTallRows), "slab gradients are for R < ", kTallRows, " rows");
  TORCH_CHECK(!g_det || slab || (!dW.has_value() && !lnw.has_value()),
              "deterministic mode: ln_linear_bwd parameter gradients need slab mode (R < 2^17 rows)");
  const int64_t sr = slab ? (R + 63) / 64 : 0;
  const int Kin = kin >= 0 ? (int)kin : (int)w.size(1);
  TORCH_CHECK(w.size(0) == N && w.is_contiguous() && w.size(1) >= Kin, "w must be (N, >= Kin) contiguous, N = g columns");
  TORCH_CHECK(x.size(0) == R && (pe.has_value() || x.size(1) == Kin), "x must be (R, Kin)");
  TORCH_CHECK(!(pe.has_value() && need_dx), "no input gradient for a split (pixels + PE) input");
  const float* pp; int prs, prows, npix; const long long* pidx;
  pe_args(pe, x, R, Kin, pp, prs, prows, npix, pe_index, pidx);
  TORCH_CHECK(Kin <= 160, "ln_linear_bwd supports Kin <= 160");
  auto f32 = g.options().dtype(torch::kFloat32);
  Tensor dx;
  float *dxp = nullptr, *dgp = nullptr, *dbp = nullptr, *dwp = nullptr, *dbiasp = nullptr;
  int vrs = -1;
  int dx_rs = Kin;
  if (need_dx && dx_out.has_value()) {
    // dX into a given (R, Kin) fp32 buffer (e.g. a parameter's gradient view); it may BE dres
    // (read and written element-wise by the same thread: dX = LN_bwd(...) + dres in place)
    CHECK_DT(*dx_out, torch::kFloat32);
    TORCH_CHECK(dx_out->dim() == 2 && dx_out->size(0) == R && dx_out->size(1) == Kin && dx_out->stride(1) == 1,
                "dx_out must be (R, Kin) rows");
    TORCH_CHECK(!dres.has_value() || dres->data_ptr() != dx_out->data_ptr() || dres->stride(0) == dx_out->stride(0),
                "dx_out aliasing dres needs the same row stride");
    dx = *dx_out; dxp = dx.data_ptr<float>(); dx_rs = (int)dx.stride(0);
  } else if (need_dx) { dx = torch::empty({R, Kin}, f32); dxp = dx.data_ptr<float>(); }
  if (lnw.has_value()) {
    TORCH_CHECK(lnb.has_value() && mean.has_value() && rstd.has_value(), "LN weight needs bias and row stats");
    TORCH_CHECK(dlnw.has_value() && dlnb.has_value(), "LN grad targets required");
    dgp = vec_target(*dlnw, Kin, "dlnw", vrs, sr);
    dbp = vec_target(*dlnb, Kin, "dlnb", vrs, sr);
  }
  int wrs = -1;  // the weight target's replica stride may differ from the vectors'
  if (dW.has_value()) dwp = vec_target(*dW, (int64_t)N * Kin, "dW", wrs, sr);
  if (db.has_value()) { TORCH_CHECK(dW.has_value(), "db needs dW"); dbiasp = vec_target(*db, N, "db", vrs, sr); }
  TORCH_CHECK(!slab || vrs < 0 || wrs < 0 || vrs == wrs, "slab targets must share one slab");
  const float* dr = nullptr; int drs = 0;
  if (dres.has_value()) { dr = f32p(*dres); drs = (int)dres->stride(0); TORCH_CHECK(dres->stride(1) == 1); }
  // very tall inputs (image K/V projections): the weight gradient leaves the row-tile kernel
  // for the streaming tall-wgrad kernel (one partial per ~R/128 rows instead of per 64)
  const bool tall = dwp != nullptr && R >= kTallRows;
  pio::ln_linear_bwd_launch(g.data_ptr(), is_bf16(g), (int)g.stride(0), N, bfp(w), (int)w.size(1), Kin, x.data_ptr(),
                            is_bf16(x), (int)x.stride(0), f32o(mean), f32o(rstd), f32o(lnw), f32o(lnb), dr, drs, dxp,
                            dx_rs, dgp, dbp, tall ? nullptr : dwp, tall ? nullptr : dbiasp, vrs < 0 ? 0 : vrs,
                            wrs < 0 ? 0 : wrs, slab ? 1 : 0, R, pp, prs, prows, npix, pidx,
                            make_job(job_slab, job_dsts, job_offs), stream());
  if (tall)
    pio::wgrad_launch(g.data_ptr(), is_bf16(g), (int)g.stride(0), N, x.data_ptr(), is_bf16(x), (int)x.stride(0), Kin,
                      lnw.has_value() ? 1 : 0, f32o(mean), f32o(rstd), f32o(lnw), f32o(lnb), R, 0, dwp, dbiasp,
                      vrs < 0 ? 0 : vrs, wrs < 0 ? 0 : wrs, pp, prs, prows, npix, pidx, stream());
  if (need_dx) return dx;
  return c10::nullopt;
}

// dW (+)= gᵀ·A', db (+)= Σ rows g  (A' = a | LN(a) | GELU(a); a may be pixels with a PE table)
void wgrad(Tensor g, Tensor a, int64_t amode, OptT mean, OptT rstd, OptT lnw, OptT lnb, int64_t rows_per_wg, Tensor dW,
           OptT db, OptT pe, int64_t kin, OptT pe_index) {
  TORCH_CHECK(g.dim() == 2 && a.dim() == 2 && g.stride(1) == 1 && a.stride(1) == 1, "2-D row tensors expected");
  const int R = (int)g.size(0), N = (int)g.size(1);
  const int Kin = kin >= 0 ? (int)kin : (int)a.size(1);
  TORCH_CHECK(a.size(0) == R, "row mismatch");
  TORCH_CHECK(pe.has_value() || a.size(1) == Kin, "a must be (R, Kin)");
  TORCH_CHECK(Kin <= 160, "wgrad supports Kin <= 160");
  TORCH_CHECK(!g_det, "deterministic mode: the streaming wgrad kernel adds partials with atomics");
  TORCH_CHECK(amode != 1 || (mean.has_value() && rstd.has_value() && lnw.has_value() && lnb.has_value()),
              "LN mode needs stats and affine");
  const float* pp; int prs, prows, npix; const long long* pidx;
  pe_args(pe, a, R, Kin, pp, prs, prows, npix, pe_index, pidx);
  int wrs = -1, vrs = -1;
  float* dwp = vec_target(dW, (int64_t)N * Kin, "dW", wrs);
  float* dbp = db.has_value() ? vec_target(*db, N, "db", vrs) : nullptr;
  pio::wgrad_launch(g.data_ptr(), is_bf16(g), (int)g.stride(0), N, a.data_ptr(), is_bf16(a), (int)a.stride(0), Kin,
                    (int)amode, f32o(mean), f32o(rstd), f32o(lnw), f32o(lnb), R, (int)rows_per_wg, dwp, dbp,
                    vrs < 0 ? 0 : vrs, wrs < 0 ? 0 : wrs, pp, prs, prows, npix, pidx, stream());
}

// per-device ticket of the CE combine kernel (its last workgroup sums the per-block partials):
// zero between launches (reset by its last taker); calls on a device are stream-ordered.
// Allocated once, so captured graphs never see it move.
constexpr int64_t kCeTickets = 4;
static Tensor& ce_ticket(const Tensor& like) {
  static std::unordered_map<int, Tensor> tickets;
  const int d = like.get_device();
  auto it = tickets.find(d);
  if (it == tickets.end()) it = tickets.emplace(d, torch::zeros({kCeTickets}, like.options().dtype(torch::kInt32))).first;
  return it->second;
}
// per-row-block arrival counters of the two-pass head's forward (re-armed by the kernel itself)
constexpr int64_t kCeRowBlockTickets = 4096;
static Tensor& ce_rb_tickets(const Tensor& like) {
  static std::unordered_map<int, Tensor> tickets;
  const int d = like.get_device();
  auto it = tickets.find(d);
  if (it == tickets.end())
    it = tickets.emplace(d, torch::zeros({kCeRowBlockTickets}, like.options().dtype(torch::kInt32))).first;
  return it->second;
}

// labels (B, L) → [idx_b (B, cap), labels_b (B, cap), gidx (gcap), glabels (gcap), total (1) fp32,
// overflow (1) bool (+ q (B, cap, C) = queries[idx_b] when the output-query array is given)]:
// per-sequence slots of the selected positions and their global compaction, one launch.
// sticky: optional persistent bool the kernel sets when this call overflows (never clears)
std::vector<Tensor> mlm_select(Tensor labels, int64_t cap, int64_t gcap, OptT sticky, OptT queries) {
  CHECK_DT(labels, torch::kInt64);
  TORCH_CHECK(labels.dim() == 2 && labels.is_contiguous(), "labels must be (B, L) contiguous");
  const int B = (int)labels.size(0), L = (int)labels.size(1);
  TORCH_CHECK(cap > 0 && cap <= L && gcap > 0 && B > 0, "bad capacities");
  auto i64 = labels.options();
  Tensor idx_b = torch::empty({B, cap}, i64), lab_b = torch::empty({B, cap}, i64);
  Tensor count = torch::empty({B}, i64.dtype(torch::kInt32));
  Tensor gidx = torch::empty({gcap}, i64), glab = torch::empty({gcap}, i64);
  Tensor total = torch::empty({1}, i64.dtype(torch::kFloat32)), ovf = torch::empty({1}, i64.dtype(torch::kBool));
  const float* P = nullptr;
  float* qp = nullptr;
  int C = 0;
  Tensor q;
  if (queries.has_value()) {
    CHECK_DT(*queries, torch::kFloat32);
    TORCH_CHECK(queries->dim() == 2 && queries->is_contiguous() && queries->size(0) >= L && queries->size(1) % 4 == 0 &&
                    queries->get_device() == labels.get_device(),
                "mlm_select: queries must be a contiguous fp32 (>= L, C) array, C % 4 == 0, on the labels' device");
    C = (int)queries->size(1);
    P = queries->data_ptr<float>();
    q = torch::empty({B, cap, C}, queries->options());
    qp = q.data_ptr<float>();
  }
  pio::mlm_select_launch(labels.data_ptr<int64_t>(), B, L, (int)cap, (int)gcap, idx_b.data_ptr<int64_t>(),
                         lab_b.data_ptr<int64_t>(), count.data_ptr<int>(), gidx.data_ptr<int64_t>(),
                         glab.data_ptr<int64_t>(), total.data_ptr<float>(), ovf.data_ptr<bool>(),
                         sticky.has_value() ? sticky->data_ptr<bool>() : nullptr, P, C, qp, stream());
  std::vector<Tensor> out{idx_b, lab_b, gidx, glab, total, ovf};
  if (queries.has_value()) out.push_back(q);
  return out;
}

static const int64_t* opt_idx(const OptT& idx, int64_t n) {
  if (!idx.has_value()) return nullptr;
  CHECK_DT(*idx, torch::kInt64);
  TORCH_CHECK(idx->is_contiguous() && idx->numel() == n, "ce: idx must hold one source row per row");
  return idx->data_ptr<int64_t>();
}

// mean CE over the rows of h (fp32 (N, C); row r = h[idx[r]] when idx is given, else h[r]) with
// label ≥ 0: → {loss (0-dim) = Σ rows / max(count, 1), per-row lse (M,), the compact bf16 rows
// hs (M, C) the backward kernels read}.  count: fp32 (1,).
// zero_out: an optional fp32 buffer the kernel clears on the way (the backward's dH accumulator)
// count_labels: count is an OUTPUT — the combine kernel writes the number of rows with a label
// ≥ 0 into it (no framework compare + reduce kernels ahead of the head; the backward reads it)
std::vector<Tensor> ce_fwd(Tensor h, OptT idx, Tensor labels, Tensor w, Tensor bias, Tensor count, OptT zero_out,
                           bool count_labels) {
  TORCH_CHECK(h.is_contiguous() && w.is_contiguous() && labels.is_contiguous() && bias.is_contiguous());
  CHECK_DT(labels, torch::kInt64);
  CHECK_DT(h, torch::kFloat32);
  CHECK_DT(count, torch::kFloat32);
  const int M = (int)labels.numel(), C = (int)h.size(1), V = (int)w.size(0);
  TORCH_CHECK(w.size(1) == C && (C == 32 || C == 64 || C == 128), "bad vocab head shape");
  TORCH_CHECK(idx.has_value() || h.size(0) == M, "ce_fwd: h must have one row per label without idx");
  const int64_t* ip = opt_idx(idx, M);
  auto f32 = h.options().dtype(torch::kFloat32);
  if (C == 64) {
    // two-pass head (ce_head.hip): the forward also forms the per-split Σ_v p·W partials of each
    // row (the hidden-state gradient up to the row-loss scale once merged); returned with the
    // splits' (max, sum) as a 4th and 5th output for ce_bwd, which merges them
    const int ns = pio::ce2_num_splits(M, V);
    Tensor pml = torch::empty({ns, M, 2}, f32), pacc = torch::empty({ns, M, C}, f32);
    Tensor picked = torch::empty({M}, f32), lse = torch::empty({M}, f32), loss = torch::empty({}, f32);
    const int nrb = pio::ce2_row_blocks(M);
    TORCH_CHECK(nrb <= kCeRowBlockTickets, "ce_fwd: too many rows for the row-block tickets");
    Tensor blk = torch::empty({2 * nrb}, f32);
    Tensor hs = torch::empty({M, C}, h.options().dtype(torch::kBFloat16));
    TORCH_CHECK(count.numel() >= 1 && count.is_contiguous(), "ce_fwd: count must hold one fp32 value");
    float* zp = nullptr;
    int64_t zn = 0;
    if (zero_out.has_value()) {
      CHECK_DT(*zero_out, torch::kFloat32);
      TORCH_CHECK(zero_out->is_contiguous() && zero_out->numel() % 4 == 0 && zero_out->get_device() == h.get_device() &&
                      reinterpret_cast<uintptr_t>(zero_out->data_ptr()) % 16 == 0,
                  "ce_fwd: zero_out must be a contiguous, 16-byte aligned fp32 buffer of 4k elements");
      zp = zero_out->data_ptr<float>();
      zn = zero_out->numel();
    }
    Tensor& tk = ce_ticket(h);
    Tensor& rbt = ce_rb_tickets(h);
    pio::ce2_fwd_launch(h.data_ptr<float>(), ip, labels.data_ptr<int64_t>(), bfp(w), f32p(bias), M, V, ns,
                        reinterpret_cast<float2*>(pml.data_ptr<float>()), pacc.data_ptr<float>(), picked.data_ptr<float>(),
                        bfp_mut(hs), lse.data_ptr<float>(), count.data_ptr<float>(), count_labels ? 1 : 0,
                        loss.data_ptr<float>(), blk.data_ptr<float>(), reinterpret_cast<unsigned*>(rbt.data_ptr<int>()),
                        reinterpret_cast<unsigned*>(tk.data_ptr<int>()), zp, zn, stream());
    checked_sync("ce_fwd");
    return {loss, lse, hs, pacc, pml};
  }
  const int ns = pio::ce_num_splits(M, V);
  Tensor part = torch::empty({ns, M, 2}, f32), picked = torch::empty({M}, f32);
  Tensor lse = torch::empty({M}, f32), loss = torch::empty({}, f32);
  Tensor blk = torch::empty({2 * pio::ce_combine_blocks(M)}, f32);
  TORCH_CHECK(count.numel() >= 1 && count.is_contiguous(), "ce_fwd: count must hold one fp32 value");
  Tensor hs = torch::empty({M, C}, h.options().dtype(torch::kBFloat16));
  Tensor& tk = ce_ticket(h);
  float* zp = nullptr;
  int64_t zn = 0;
  if (zero_out.has_value()) {
    CHECK_DT(*zero_out, torch::kFloat32);
    TORCH_CHECK(zero_out->is_contiguous() && zero_out->numel() % 4 == 0 && zero_out->get_device() == h.get_device() &&
                    reinterpret_cast<uintptr_t>(zero_out->data_ptr()) % 16 == 0,
                "ce_fwd: zero_out must be a contiguous, 16-byte aligned fp32 buffer of 4k elements");
    zp = zero_out->data_ptr<float>();
    zn = zero_out->numel();
  }
  pio::ce_fwd_launch(C, h.data_ptr<float>(), ip, labels.data_ptr<int64_t>(), bfp(w), f32p(bias), M, V,
                     part.data_ptr<float>(), picked.data_ptr<float>(), lse.data_ptr<float>(), count.data_ptr<float>(),
                     loss.data_ptr<float>(), blk.data_ptr<float>(), reinterpret_cast<unsigned*>(tk.data_ptr<int>()),
                     bfp_mut(hs), ns, zp, zn, count_labels ? 1 : 0, stream());
  checked_sync("ce_fwd");
  return {loss, lse, hs};
}

// h: the compact bf16 rows from ce_fwd.  dH (+)= rows: row r lands in dH[rowmap[r]] when rowmap
// is given (dH then has the full (positions, C) shape), else in dH[r]; dW / db accumulate or
// overwrite.  The row-loss gradient
// is gout / max(count, 1) (gout: the 0-dim gradient of the mean loss).
// slab: the dW kernel stores its row-split partials into a returned (splits, V·C + V₄) slab
// instead of adding them (the caller sums it into dW | db with a slab job, offsets 0 and V·C).
OptT ce_bwd(Tensor h, Tensor labels, Tensor w, Tensor bias, Tensor lse, Tensor gout, Tensor count, Tensor dH,
            Tensor dW, Tensor db, bool accumulate, OptT rowmap, bool slab, OptT u, OptT u_ml) {
  const int M = (int)labels.numel(), C = (int)h.size(1), V = (int)w.size(0);
  CHECK_DT(h, torch::kBFloat16);
  TORCH_CHECK(h.size(0) == M, "ce_bwd: h must be the compact (M, C) bf16 rows of ce_fwd");
  CHECK_DT(gout, torch::kFloat32);
  CHECK_DT(count, torch::kFloat32);
  TORCH_CHECK(h.is_contiguous() && dH.is_contiguous() && dW.is_contiguous() && db.is_contiguous());
  TORCH_CHECK(dH.dim() == 2 && dH.size(1) == C, "dH must be (rows, C)");
  const int64_t* rm = nullptr;
  if (rowmap.has_value()) {
    CHECK_DT(*rowmap, torch::kInt64);
    TORCH_CHECK(rowmap->is_contiguous() && rowmap->numel() == M, "rowmap must hold one row index per row");
    rm = rowmap->data_ptr<int64_t>();
  } else {
    TORCH_CHECK(dH.size(0) == M, "dH must be (M, C) without a rowmap");
  }
  Tensor sl;
  if (u.has_value()) {  // the two-pass head's backward: dW / db pass + the dH rows g·u
    // u: the forward's per-split Σ p·W partials (splits, M, 64), u_ml: their (max, sum) (splits, M, 2)
    CHECK_DT(*u, torch::kFloat32);
    TORCH_CHECK(u_ml.has_value(), "ce_bwd: the two-pass head needs the split (max, sum) pairs");
    CHECK_DT(*u_ml, torch::kFloat32);
    TORCH_CHECK(C == 64 && u->is_contiguous() && u->dim() == 3 && u->size(1) == M && u->size(2) == C &&
                    u_ml->is_contiguous() && u_ml->dim() == 3 && u_ml->size(0) == u->size(0) && u_ml->size(1) == M &&
                    u_ml->size(2) == 2 && u->size(0) <= 16,
                "ce_bwd: u must be (splits, M, 64) and u_ml (splits, M, 2) fp32");
    if (slab) sl = torch::empty({pio::ce2_bwd_splits(M, V), (int64_t)V * C + ((V + 3) & ~3)}, dW.options());
    pio::ce2_bwd_launch(bfp(h), labels.data_ptr<int64_t>(), bfp(w), f32p(bias), f32p(lse), u->data_ptr<float>(),
                        reinterpret_cast<const float2*>(u_ml->data_ptr<float>()), (int)u->size(0), f32p(gout),
                        f32p(count), M, V, dW.data_ptr<float>(), db.data_ptr<float>(),
                        slab ? sl.data_ptr<float>() : nullptr, accumulate ? 1 : 0, dH.data_ptr<float>(), dH.size(0), rm,
                        stream());
    if (slab) return sl;
    return c10::nullopt;
  }
  if (slab) sl = torch::empty({pio::ce_dw_splits(M, V), (int64_t)V * C + ((V + 3) & ~3)}, dW.options());
  pio::ce_bwd_launch(C, bfp(h), labels.data_ptr<int64_t>(), bfp(w), f32p(bias), f32p(lse), f32p(gout),
                     f32p(count), M, V, dH.data_ptr<float>(), dH.size(0), rm, dW.data_ptr<float>(), db.data_ptr<float>(),
                     accumulate ? 1 : 0, slab ? sl.data_ptr<float>() : nullptr, g_det ? 1 : 0, stream());
  if (slab) return sl;
  return c10::nullopt;
}

Tensor embed_fwd(Tensor ids, Tensor E, Tensor P, double scale) {
  TORCH_CHECK(ids.is_contiguous() && E.is_contiguous() && P.is_contiguous());
  CHECK_DT(ids, torch::kInt64);
  const long long rows = ids.numel();
  const int L = (int)ids.size(1), C = (int)E.size(1);
  TORCH_CHECK(C % 4 == 0, "embedding width must be a multiple of 4");
  Tensor out = torch::empty({ids.size(0), L, C}, E.options());
  pio::embed_fwd_launch(ids.data_ptr<int64_t>(), f32p(E), f32p(P), out.data_ptr<float>(), rows, L, C, (float)scale,
                        E.size(0), stream());
  checked_sync("embed_fwd");
  return out;
}

void embed_bwd(Tensor ids, Tensor g, OptT dE, OptT dP, double scale, OptT job_slab, std::vector<Tensor> job_dsts,
               std::vector<int64_t> job_offs) {
  TORCH_CHECK(g.is_contiguous() && ids.is_contiguous());
  const pio::SlabJob job = make_job(job_slab, job_dsts, job_offs);
  const int B = (int)ids.size(0), L = (int)ids.size(1), C = (int)g.size(2);
  if (dE.has_value()) TORCH_CHECK(dE->is_contiguous() && dE->size(1) == C, "dE must be (V, C) contiguous");
  if (dP.has_value()) TORCH_CHECK(dP->is_contiguous() && dP->size(1) == C && dP->size(0) >= L, "dP must be (>= L, C)");
  // one launch: block-local sort + run folding for dE, batch sums for dP (C ∈ {64, 128, 256}, ids < 2^24)
  if ((!dE.has_value() || dE->size(0) < (1 << 24)) &&
      pio::embed_bwd_local_launch(ids.data_ptr<int64_t>(), f32p(g), dE.has_value() ? dE->data_ptr<float>() : nullptr,
                                  dP.has_value() ? dP->data_ptr<float>() : nullptr, B, L, C, (float)scale, job,
                                  stream()))
    return;
  if (job.slab) pio::slab_reduce_launch(job, stream());  // the fallback paths carry no job
  if (dE.has_value()) {  // token-embedding rows: sort positions by id, fold equal-id runs, then add
    TORCH_CHECK(dE->is_contiguous() && dE->size(1) == C, "dE must be (V, C) contiguous");
    const bool small = dE->size(0) <= 32767;  // int16 keys: a 2-pass radix sort instead of 8
    Tensor keys = small ? ids.reshape({-1}).to(torch::kInt16) : ids.reshape({-1});
    auto sorted = keys.sort();
    Tensor sid = std::get<0>(sorted).to(torch::kInt64).contiguous(), perm = std::get<1>(sorted).contiguous();
    pio::embed_bwd_sorted_launch(sid.data_ptr<int64_t>(), perm.data_ptr<int64_t>(), f32p(g), dE->data_ptr<float>(),
                                 ids.numel(), C, (float)scale, stream());
  }
  if (dP.has_value())
    pio::embed_bwd_launch(ids.data_ptr<int64_t>(), f32p(g), nullptr, dP->data_ptr<float>(), B, L, C, (float)scale,
                          stream());
}

// state: int64 (3,) {seed, counter, ticket} on the device (see text_mask_kernel); advance: the
// launch increments the counter (fresh masks on every call / graph replay)
std::vector<Tensor> text_mask(Tensor x, OptT pad, Tensor state, int64_t unk, int64_t mask, double p, int64_t lo,
                              int64_t hi, bool advance) {
  TORCH_CHECK(x.is_contiguous() && state.is_contiguous() && state.numel() == 3, "text_mask: bad x / state");
  CHECK_DT(x, torch::kInt64);
  CHECK_DT(state, torch::kInt64);
  TORCH_CHECK(hi > lo && hi - lo < (1LL << 32), "text_mask: bad random-id range");
  const long long n = x.numel();
  TORCH_CHECK(n < (1LL << 32), "text_mask: too many tokens");
  Tensor xm = torch::empty_like(x), lab = torch::empty_like(x);
  const bool* pp = nullptr;
  if (pad.has_value()) {
    CHECK_DT(*pad, torch::kBool);
    TORCH_CHECK(pad->is_contiguous() && pad->numel() == n, "text_mask: pad mask must match x");
    pp = pad->data_ptr<bool>();
  }
  pio::text_mask_launch(x.data_ptr<int64_t>(), pp, state.data_ptr<int64_t>(), xm.data_ptr<int64_t>(),
                        lab.data_ptr<int64_t>(), n, (int)unk, (int)mask, (float)p, (int)lo, (uint32_t)(hi - lo),
                        advance ? 1 : 0, stream());
  return {xm, lab};
}

// one launch per replayed step: dsts[i] <- srcs[i] (same device, dtype-agnostic byte copies of
// contiguous tensors of equal size) and hyper_dst[:len(hyper)] <- hyper (values by kernel argument)
// seed_dst + seeds: a captured step's dropout seed slots (int64, ≤ 64 values) written in the same launch
void stage_step(std::vector<Tensor> dsts, std::vector<Tensor> srcs, OptT hyper_dst, std::vector<double> hyper,
                OptT seed_dst, std::vector<int64_t> seeds) {
  TORCH_CHECK(dsts.size() == srcs.size() && dsts.size() <= 8 && hyper.size() <= 8, "stage_step: at most 8 tensors / 8 values");
  std::vector<void*> d;
  std::vector<const void*> x;
  std::vector<long long> n;
  for (size_t i = 0; i < dsts.size(); ++i) {
    const Tensor& a = dsts[i];
    const Tensor& b = srcs[i];
    TORCH_CHECK(a.is_cuda() && b.is_cuda() && a.get_device() == b.get_device() && a.is_contiguous() && b.is_contiguous() &&
                    a.scalar_type() == b.scalar_type() && a.numel() == b.numel(),
                "stage_step: pairs must be contiguous same-device tensors of equal dtype and size");
    d.push_back(a.data_ptr());
    x.push_back(b.data_ptr());
    n.push_back((long long)(a.numel() * a.element_size()));
  }
  float* hp = nullptr;
  std::vector<float> hv(hyper.begin(), hyper.end());
  if (hyper_dst.has_value()) {
    CHECK_DT(*hyper_dst, torch::kFloat32);
    TORCH_CHECK(hyper_dst->is_contiguous() && hyper_dst->numel() >= (int64_t)hv.size(), "stage_step: hyper_dst too small");
    hp = hyper_dst->data_ptr<float>();
  }
  long long* sp = nullptr;
  if (!seeds.empty()) {
    TORCH_CHECK(seed_dst.has_value() && seed_dst->is_cuda() && seed_dst->is_contiguous() &&
                    seed_dst->scalar_type() == torch::kInt64 && seed_dst->numel() >= (int64_t)seeds.size() &&
                    seeds.size() <= 64,
                "stage_step: seed_dst must be a contiguous int64 device tensor of >= len(seeds) (<= 64) slots");
    sp = reinterpret_cast<long long*>(seed_dst->data_ptr<int64_t>());
  }
  std::vector<long long> sv(seeds.begin(), seeds.end());
  TORCH_CHECK(pio::stage_step_launch(d.data(), x.data(), n.data(), (int)d.size(), hp, hv.data(), (int)hv.size(), sp,
                                     sv.data(), (int)sv.size(), stream()) == 0);
}

// Σ g² as kSumsqBlocks fixed-order partials (part: ≥ kSumsqBlocks fp32), read by adamw(norm_part=)
constexpr int kSumsqParts = 512;  // common.h kSumsqBlocks
void sumsq(Tensor g, Tensor part) {
  CHECK_DT(g, torch::kFloat32); CHECK_DT(part, torch::kFloat32);
  TORCH_CHECK(g.is_contiguous() && part.is_contiguous() && part.numel() >= kSumsqParts,
              "sumsq: contiguous gradient, a contiguous partial buffer of >= 512 floats");
  pio::sumsq_launch(f32p(g), g.numel(), part.data_ptr<float>(), stream());
}

// a, b: (B, ...) fp32 contiguous, equal shapes → (Σ_b a[b], Σ_b b[b]) in one launch
// oa = Σ_b a[b] (a optional), ob = Σ_b b[b] — or, with ob_acc, ob_acc += Σ_b b[b] in place (the
// gradient of a batch-broadcast parameter straight into its gradient buffer)
std::vector<Tensor> batch_sum2(OptT a, Tensor b, OptT ob_acc) {
  CHECK_DT(b, torch::kFloat32);
  TORCH_CHECK(b.is_contiguous() && b.dim() >= 2, "batch_sum2: b must be contiguous (B, ...)");
  const long long n = b.numel() / b.size(0);
  TORCH_CHECK(n % 4 == 0 && reinterpret_cast<uintptr_t>(b.data_ptr()) % 16 == 0, "batch_sum2: 16-byte rows");
  if (a.has_value()) {
    CHECK_DT(*a, torch::kFloat32);
    TORCH_CHECK(a->is_contiguous() && a->sizes() == b.sizes() && reinterpret_cast<uintptr_t>(a->data_ptr()) % 16 == 0,
                "batch_sum2: a must match b");
  }
  std::vector<int64_t> shp(b.sizes().begin() + 1, b.sizes().end());
  Tensor oa = a.has_value() ? torch::empty(shp, b.options()) : Tensor();
  Tensor ob;
  if (ob_acc.has_value()) {
    CHECK_DT(*ob_acc, torch::kFloat32);
    TORCH_CHECK(ob_acc->is_contiguous() && ob_acc->numel() == n && reinterpret_cast<uintptr_t>(ob_acc->data_ptr()) % 16 == 0,
                "batch_sum2: ob_acc must be a contiguous, 16-byte aligned tensor of one batch element's size");
    ob = ob_acc->view(shp);
  } else {
    ob = torch::empty(shp, b.options());
  }
  pio::batch_sum2_launch(a.has_value() ? a->data_ptr<float>() : nullptr, b.data_ptr<float>(),
                         a.has_value() ? oa.data_ptr<float>() : nullptr, ob.data_ptr<float>(), (int)b.size(0), n, n,
                         ob_acc.has_value() ? 1 : 0, stream());
  return {oa, ob};
}

// dst (N, C) fp32 += src (R, C) fp32 scattered to rows idx (R) — the backward of a row gather
void index_add_rows(Tensor dst, Tensor idx, Tensor src) {
  CHECK_DT(dst, torch::kFloat32); CHECK_DT(src, torch::kFloat32); CHECK_DT(idx, torch::kInt64);
  TORCH_CHECK(dst.dim() == 2 && dst.is_contiguous() && src.dim() == 2 && src.is_contiguous() && idx.is_contiguous(),
              "index_add_rows: contiguous dst (N, C), src (R, C), idx (R)");
  TORCH_CHECK(src.size(1) == dst.size(1) && idx.numel() == src.size(0) && dst.size(1) % 4 == 0,
              "index_add_rows: shapes (C % 4 == 0)");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(dst.data_ptr()) % 16 == 0 && reinterpret_cast<uintptr_t>(src.data_ptr()) % 16 == 0,
              "index_add_rows: 16-byte aligned rows");
  if (src.size(0) == 0) return;
  pio::index_add_rows_launch(dst.data_ptr<float>(), dst.size(0), idx.data_ptr<int64_t>(), f32p(src), src.size(0),
                             (int)src.size(1), stream());
  checked_sync("index_add_rows");
}

// src (N, C) fp32 rows at idx (R) → (R, C) — a row gather (decoder output queries of a sparse image)
Tensor gather_rows(Tensor src, Tensor idx) {
  CHECK_DT(src, torch::kFloat32); CHECK_DT(idx, torch::kInt64);
  TORCH_CHECK(src.dim() == 2 && src.is_contiguous() && idx.is_contiguous() && src.size(1) % 4 == 0 &&
                  reinterpret_cast<uintptr_t>(src.data_ptr()) % 16 == 0,
              "gather_rows: contiguous 16-byte aligned src (N, C), C % 4 == 0, contiguous idx");
  Tensor out = torch::empty({idx.numel(), src.size(1)}, src.options());
  if (idx.numel() == 0) return out;
  pio::gather_rows_launch(out.data_ptr<float>(), f32p(src), src.size(0), idx.data_ptr<int64_t>(), idx.numel(),
                          (int)src.size(1), stream());
  checked_sync("gather_rows");
  return out;
}

namespace {
void check_pixel_head(const Tensor& h, const Tensor& w, const Tensor& b, const Tensor& labels, const Tensor& wts) {
  CHECK_DT(h, torch::kFloat32); CHECK_DT(w, torch::kFloat32); CHECK_DT(b, torch::kFloat32);
  CHECK_DT(labels, torch::kInt64); CHECK_DT(wts, torch::kFloat32);
  TORCH_CHECK(h.dim() == 2 && h.is_contiguous() && w.dim() == 2 && w.is_contiguous() && b.is_contiguous() &&
                  labels.is_contiguous() && wts.is_contiguous(), "pixel head: contiguous h (R, C), w (K, C)");
  const int C = (int)h.size(1), K = (int)w.size(0);
  TORCH_CHECK((C == 32 || C == 64 || C == 128) && K >= 2 && K <= 4 && w.size(1) == C && b.numel() == K &&
                  wts.numel() == K && labels.numel() == h.size(0), "pixel head: C in {32, 64, 128}, 2 <= K <= 4");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(h.data_ptr()) % 16 == 0 && reinterpret_cast<uintptr_t>(w.data_ptr()) % 16 == 0,
              "pixel head: 16-byte aligned rows");
}
}  // namespace

// → [stats (4 + 2K sums: Σ w·ce, Σ w, n(lab>0), hit(lab>0), (n_k, hit_k)… | acc, acc_1 … acc_{K-1}),
//    loss = Σ w·ce / Σ w (0-dim)]
std::vector<Tensor> pixel_ce_fwd(Tensor h, Tensor w, Tensor b, Tensor labels, Tensor wts) {
  check_pixel_head(h, w, b, labels, wts);
  const long long R = h.size(0);
  const int K = (int)w.size(0);
  // every block of the launch stores its whole partial row (zeros only for an empty input)
  Tensor part = R > 0 ? torch::empty({pio::pixel_ce_blocks(R), 4 + 2 * K}, h.options())
                      : torch::zeros({pio::pixel_ce_blocks(R), 4 + 2 * K}, h.options());
  Tensor stats = torch::empty({4 + 2 * K + K}, h.options()), loss = torch::empty({}, h.options());
  pio::pixel_ce_fwd_launch((int)h.size(1), K, f32p(h), f32p(w), f32p(b), labels.data_ptr<int64_t>(), f32p(wts), R,
                           part.data_ptr<float>(), stats.data_ptr<float>(), loss.data_ptr<float>(), stream());
  return {stats, loss};
}

// dH (R, C) written; dW (K, C) / db (K) += the head's weight gradients (fixed-order sums)
void pixel_ce_bwd(Tensor h, Tensor w, Tensor b, Tensor labels, Tensor wts, Tensor gout, Tensor stats, Tensor dH,
                  Tensor dW, Tensor db) {
  check_pixel_head(h, w, b, labels, wts);
  CHECK_DT(gout, torch::kFloat32); CHECK_DT(stats, torch::kFloat32); CHECK_DT(dH, torch::kFloat32);
  CHECK_DT(dW, torch::kFloat32); CHECK_DT(db, torch::kFloat32);
  TORCH_CHECK(dH.is_contiguous() && dH.sizes() == h.sizes() && gout.numel() == 1 && stats.numel() >= 2,
              "pixel head bwd: dH like h, scalar loss gradient");
  TORCH_CHECK(dW.is_contiguous() && dW.numel() == w.numel() && db.is_contiguous() && db.numel() == b.numel(),
              "pixel head bwd: dW / db like w / b");
  const long long R = h.size(0);
  const int K = (int)w.size(0), C = (int)h.size(1);
  Tensor part = R > 0 ? torch::empty({pio::pixel_ce_blocks(R), (int64_t)K * C + K}, h.options())
                      : torch::zeros({pio::pixel_ce_blocks(R), (int64_t)K * C + K}, h.options());
  pio::pixel_ce_bwd_launch(C, K, f32p(h), f32p(w), f32p(b), labels.data_ptr<int64_t>(), f32p(wts), f32p(gout),
                           f32p(stats), R, dH.data_ptr<float>(), part.data_ptr<float>(), dW.data_ptr<float>(),
                           db.data_ptr<float>(), stream());
}

void adamw(Tensor p, Tensor g, Tensor m, Tensor v, OptT shadow, Tensor hyper, double eps, double wd, double clip,
           double gscale, bool l2, bool zero_grad, OptT loss_src, OptT loss_ring, OptT norm_part) {
  TORCH_CHECK(clip <= 0 || (norm_part.has_value() && norm_part->is_contiguous() && norm_part->numel() >= kSumsqParts &&
                            norm_part->scalar_type() == torch::kFloat32),
              "adamw: clip > 0 needs norm_part (the sumsq partials of the gradient)");
  TORCH_CHECK(p.is_contiguous() && g.is_contiguous() && m.is_contiguous() && v.is_contiguous());
  TORCH_CHECK(p.numel() == g.numel() && p.numel() == m.numel() && p.numel() == v.numel());
  uint16_t* sp = nullptr;
  if (shadow.has_value()) { TORCH_CHECK(shadow->numel() == p.numel()); sp = reinterpret_cast<uint16_t*>(shadow->data_ptr()); }
  TORCH_CHECK(loss_src.has_value() == loss_ring.has_value(), "adamw: loss_src and loss_ring go together");
  if (loss_src.has_value()) {
    CHECK_DT(*loss_src, torch::kFloat32); CHECK_DT(*loss_ring, torch::kFloat32);
    TORCH_CHECK(loss_src->numel() == 1 && loss_ring->is_contiguous() && loss_ring->numel() >= 1 && hyper.numel() >= 8,
                "adamw: scalar loss_src, contiguous loss_ring, hyper[7] = ring slot");
  }
  pio::adamw_launch(p.data_ptr<float>(), g.data_ptr<float>(), m.data_ptr<float>(), v.data_ptr<float>(), sp, p.numel(),
                    f32p(hyper), (float)eps, (float)wd, (float)clip, (float)gscale, l2 ? 1 : 0, zero_grad ? 1 : 0,
                    loss_src.has_value() ? f32p(*loss_src) : nullptr,
                    loss_ring.has_value() ? loss_ring->data_ptr<float>() : nullptr,
                    loss_ring.has_value() ? (int)loss_ring->numel() : 1,
                    clip > 0 ? f32p(*norm_part) : nullptr, stream());
}

// self-test of the device cross-lane reductions: (6, 64) = wave_sum, wave_max, half_sum,
// half_max, xor16_sum, xor32_sum of a 64-element fp32 vector
Tensor reduce_probe(Tensor x) {
  TORCH_CHECK(x.is_contiguous() && x.numel() == 64, "reduce_probe takes 64 floats");
  Tensor out = torch::empty({6, 64}, x.options().dtype(torch::kFloat32));
  pio::reduce_probe_launch(f32p(x), out.data_ptr<float>(), stream());
  return out;
}

// grad[:n] += Σ_r rep[r], rep ← 0   (rep: (R, n) contiguous fp32)
void fold_replicas(Tensor grad, Tensor rep) {
  CHECK_DT(grad, torch::kFloat32); CHECK_DT(rep, torch::kFloat32);
  TORCH_CHECK(rep.dim() == 2 && rep.is_contiguous() && grad.is_contiguous() && grad.numel() >= rep.size(1),
              "fold_replicas: rep must be (R, n) contiguous, grad at least n long");
  if (rep.size(1) == 0) return;
  pio::fold_replicas_launch(grad.data_ptr<float>(), rep.data_ptr<float>(), rep.size(1), (int)rep.size(0), stream());
}

// standalone slab job (see make_job)
void slab_reduce(Tensor slab, std::vector<Tensor> dsts, std::vector<int64_t> offs) {
  pio::slab_reduce_launch(make_job(slab, dsts, offs), stream());
}

void cast_bf16(Tensor x, Tensor y) {
  TORCH_CHECK(x.is_contiguous() && y.is_contiguous() && x.numel() == y.numel());
  pio::cast_bf16_launch(f32p(x), reinterpret_cast<uint16_t*>(y.data_ptr()), x.numel(), stream());
}

// factored LN + K/V projection over [pixels ‖ PE] (pe_proj.hip).  pix (R, nc) with R = B·M,
// P (M, O) = (E⊙γ_e)·W_eᵀ, pes/pesq (M), wpg (nc, O), gw/bw (O) → y bf16 (R, O), mean/rstd (R)
std::vector<Tensor> pe_proj_fwd(Tensor pix, Tensor P, Tensor pes, Tensor pesq, Tensor wpg, Tensor gw, Tensor bw,
                                int64_t kin, double eps) {
  for (const Tensor* t : {&pix, &P, &pes, &pesq, &wpg, &gw, &bw}) {
    CHECK_CUDA(*t); CHECK_DT(*t, torch::kFloat32);
    TORCH_CHECK(t->is_contiguous(), "pe_proj_fwd: operands must be contiguous");
  }
  TORCH_CHECK(pix.dim() == 2 && P.dim() == 2, "pe_proj_fwd: pix (R, nc), P (M, O)");
  const long long R = pix.size(0);
  const int nc = (int)pix.size(1), M = (int)P.size(0), O = (int)P.size(1);
  TORCH_CHECK(nc >= 1 && nc <= 4 && O % 4 == 0 && O <= 512 && M > 0 && R % M == 0 && kin > nc,
              "pe_proj_fwd: need 1 <= nc <= 4, O % 4 == 0, O <= 512, R a multiple of M");
  TORCH_CHECK(pes.numel() == M && pesq.numel() == M && wpg.size(0) == nc && wpg.size(1) == O && gw.numel() == O &&
                  bw.numel() == O, "pe_proj_fwd: operand shapes");
  auto y = torch::empty({R, O}, pix.options().dtype(torch::kBFloat16));
  auto mean = torch::empty({R}, pix.options());
  auto rstd = torch::empty({R}, pix.options());
  if (R > 0)
    pio::pe_proj_fwd_launch(f32p(pix), nc, f32p(P), f32p(pes), f32p(pesq), f32p(wpg), f32p(gw), f32p(bw), R, M, O,
                            (int)kin, (float)eps, bfp_mut(y), mean.data_ptr<float>(), rstd.data_ptr<float>(), stream());
  return {y, mean, rstd};
}

// C (M, N) fp32 (bf16 if bf16_out) = A (M, K) bf16 · B (N, K) bf16ᵀ — the factored projection's
// per-step PE GEMM
Tensor pe_gemm(Tensor A, Tensor B, bool bf16_out, int64_t pad_rows) {
  CHECK_CUDA(A); CHECK_DT(A, torch::kBFloat16); CHECK_DT(B, torch::kBFloat16);
  TORCH_CHECK(A.dim() == 2 && B.dim() == 2 && A.is_contiguous() && B.is_contiguous() && A.size(1) == B.size(1),
              "pe_gemm: A (M, K), B (N, K) contiguous");
  const int M = (int)A.size(0), N = (int)B.size(0), K = (int)A.size(1);
  TORCH_CHECK(K % 32 == 0 && N % 128 == 0 && K > 0, "pe_gemm: K a multiple of 32, N a multiple of 128");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(A.data_ptr()) % 16 == 0 && reinterpret_cast<uintptr_t>(B.data_ptr()) % 16 == 0,
              "pe_gemm: 16-byte aligned operands");
  TORCH_CHECK(pad_rows >= 0, "pe_gemm: pad_rows >= 0");
  Tensor C = torch::empty({M + pad_rows, N}, A.options().dtype(bf16_out ? torch::kBFloat16 : torch::kFloat32));
  // the zero rows past M (read by prefetches, never used) are written by the GEMM launch itself
  if (M + pad_rows > 0) pio::pe_gemm_launch(bfp(A), bfp(B), C.data_ptr(), bf16_out, M, N, K, (int)(M + pad_rows), stream());
  return C;
}

// weight / LayerNorm gradients of the factored projection, ADDED into the given targets (each
// optional, fp32 contiguous): D (M, O) = Σ_b dY·rσ, part (nblk, (2 + nc)·O) = [ΣdY | ΣdY·μ·rσ |
// ΣdY·x̂_c] partial rows, E (M, Kp) the bf16 PE table, W = [Wa; Wb] (O, kin) as two row blocks
void pe_grads(Tensor D, Tensor part, Tensor E, Tensor Wa, Tensor Wb, Tensor g, Tensor b, int64_t nc, OptT dWa, OptT dWb,
              OptT db, OptT dg, OptT dbeta) {
  for (const Tensor* t : {&D, &part, &Wa, &Wb, &g, &b}) {
    CHECK_CUDA(*t); CHECK_DT(*t, torch::kFloat32);
    TORCH_CHECK(t->is_contiguous(), "pe_grads: contiguous operands");
  }
  CHECK_DT(E, torch::kBFloat16);
  TORCH_CHECK(E.is_contiguous() && E.dim() == 2 && D.dim() == 2 && E.size(0) == D.size(0), "pe_grads: E (M, Kp), D (M, O)");
  const int M = (int)D.size(0), O = (int)D.size(1), Kp = (int)E.size(1), kin = (int)g.numel(), Ch = (int)Wa.size(0);
  const int on = O % 128 == 0 ? 128 : O;  // output columns per workgroup (pe_grads_launch)
  TORCH_CHECK(Kp % 32 == 0 && Kp <= 384 && O % 32 == 0 && on <= 256 && (Kp / 32) * (on / 32) <= 36 && kin <= Kp,
              "pe_grads: Kp a multiple of 32 (≤ 384), O a multiple of 128 or ≤ 256, ≤ 36 output tiles per group");
  TORCH_CHECK(Wa.size(1) == kin && Wb.size(1) == kin && Ch + Wb.size(0) == O && b.numel() == kin, "pe_grads: W shapes");
  TORCH_CHECK(part.size(1) == (2 + nc) * O, "pe_grads: part width");
  auto tgt = [](const OptT& t, int64_t n, const char* name) -> float* {
    if (!t.has_value()) return nullptr;
    CHECK_DT(*t, torch::kFloat32);
    TORCH_CHECK(t->is_contiguous() && t->numel() == n, "pe_grads: target ", name);
    return t->data_ptr<float>();
  };
  pio::PeGradTargets tg{tgt(dWa, (int64_t)Ch * kin, "dWa"), tgt(dWb, (int64_t)(O - Ch) * kin, "dWb"), tgt(db, O, "db"),
                        tgt(dg, kin, "dg"), tgt(dbeta, kin, "dbeta")};
  const int S = pio::pe_grad_splits(M);
  auto f32 = D.options();
  Tensor slab = torch::empty({S, Kp, O}, f32), graw = torch::empty({Kp, O}, f32), tot = torch::empty({(2 + nc) * O}, f32);
  pio::pe_grads_launch(bfp(E), D.data_ptr<float>(), M, Kp, O, part.data_ptr<float>(), (int)part.size(0),
                       slab.data_ptr<float>(), graw.data_ptr<float>(), tot.data_ptr<float>(), Wa.data_ptr<float>(),
                       Wb.data_ptr<float>(), g.data_ptr<float>(), b.data_ptr<float>(), Ch, kin, (int)nc, tg, stream());
}

// W (O, kin) fp32 — or the row blocks W (O1, kin) and W2 (O − O1, kin) of a separate K / V pair,
// never concatenated — γ/β (kin), bias (O) → [Wg (O, Kp) bf16 = W⊙γ on columns [nc, kin) else 0,
// wpg (nc, O) = (W⊙γ)[:, :nc]ᵀ, gw (O) = W·γ, bw (O) = W·β + bias]
std::vector<Tensor> pe_weight_prep(Tensor W, Tensor g, Tensor b, Tensor bias, int64_t nc, int64_t Kp, OptT W2) {
  for (const Tensor* t : {&W, &g, &b, &bias}) {
    CHECK_CUDA(*t); CHECK_DT(*t, torch::kFloat32);
    TORCH_CHECK(t->is_contiguous(), "pe_weight_prep: contiguous operands");
  }
  const int O1 = (int)W.size(0), kin = (int)W.size(1);
  if (W2.has_value()) {
    CHECK_CUDA(*W2); CHECK_DT(*W2, torch::kFloat32);
    TORCH_CHECK(W2->is_contiguous() && W2->dim() == 2 && W2->size(1) == kin, "pe_weight_prep: W2 (O2, kin) contiguous");
  }
  const int O = O1 + (W2.has_value() ? (int)W2->size(0) : 0);
  TORCH_CHECK(g.numel() == kin && b.numel() == kin && bias.numel() == O && nc >= 1 && nc < kin && Kp >= kin,
              "pe_weight_prep: shapes");
  auto f32 = W.options();
  Tensor Wg = torch::empty({O, Kp}, f32.dtype(torch::kBFloat16));
  Tensor wpg = torch::empty({nc, O}, f32), gw = torch::empty({O}, f32), bw = torch::empty({O}, f32);
  Tensor wt = torch::empty({6, O}, f32);  // implicit-K/V generation table (attention_pe.hip)
  TORCH_CHECK(nc <= 4, "pe_weight_prep: at most 4 pixel channels");
  pio::pe_weight_prep_launch(W.data_ptr<float>(), W2.has_value() ? W2->data_ptr<float>() : nullptr, O1,
                             g.data_ptr<float>(), b.data_ptr<float>(), bias.data_ptr<float>(), O,
                             (int)nc, kin, (int)Kp, bfp_mut(Wg), wpg.data_ptr<float>(), gw.data_ptr<float>(),
                             bw.data_ptr<float>(), wt.data_ptr<float>(), stream());
  return {Wg, wpg, gw, bw, wt};
}

// backward pass over dY (R, O): D (M, O) and per-block partials (nblk, (2 + nc)·O) of
// [Σ dY | Σ dY·μ·rσ | Σ dY·x̂_c (c < nc)]
std::vector<Tensor> pe_proj_bwd(Tensor dy, Tensor pix, Tensor mean, Tensor rstd, int64_t M) {
  for (const Tensor* t : {&dy, &pix, &mean, &rstd}) {
    CHECK_CUDA(*t); CHECK_DT(*t, torch::kFloat32);
    TORCH_CHECK(t->is_contiguous(), "pe_proj_bwd: operands must be contiguous");
  }
  TORCH_CHECK(dy.dim() == 2 && pix.dim() == 2 && dy.size(0) == pix.size(0), "pe_proj_bwd: dy (R, O), pix (R, nc)");
  const long long R = dy.size(0);
  const int nc = (int)pix.size(1), O = (int)dy.size(1);
  TORCH_CHECK(M > 0 && R % M == 0 && R / M <= INT32_MAX && nc >= 1 && nc <= 4 && O % 4 == 0 && O <= 512 &&
                  mean.numel() == R && rstd.numel() == R, "pe_proj_bwd: shapes");
  const int nblk = pio::pe_proj_bwd_blocks((int)M);
  auto D = torch::empty({M, O}, dy.options());
  auto part = torch::empty({nblk, (2 + nc) * O}, dy.options());
  pio::pe_proj_bwd_launch(f32p(dy), f32p(pix), nc, f32p(mean), f32p(rstd), (int)(R / M), (int)M, O,
                          D.data_ptr<float>(), part.data_ptr<float>(), stream());
  return {D, part};
}

// encoder cross-attention backward fused with the factored K/V-projection reductions
// (attention_pe.hip): queries (1 | B, Nq ≤ 32, ·), head dim 32, no key mask, no dropout.
// Writes dq (zeroed here) — (Nq, C) summed over the batch for broadcast queries, else (B, Nq, C)
// — and D (M, 2C), part (nkb·bsplit, (2 + nc)·2C), both added onto when accumulate.
// implicit K/V (impl != null): kv / mean / rstd are absent; the factored kernel works from P' (M, 2C)
// bf16, the PE row sums pes / pesq (M) and the per-column table wt (6, 2C) of pe_weight_prep
struct PeImplicit { Tensor P, pes, pesq, wt; double kin, eps; };

// persistent mode of the PE attention backward (attention_pe.hip): one workgroup per CU over
// (key block, head, batch group) items when there are at least as many pairs as CUs
static int pe_bwd_slots(int M, int H, int64_t bsplit) {
  if (g_det || bsplit != 1) return 0;
  int dev = 0, ncu = 256;
  (void)hipGetDevice(&dev);
  (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
  const int nkb = (M + 255) / 256;
  return (int64_t)nkb * H >= ncu ? ncu : 0;
}

// rows of the `part` buffer the PE attention backward writes for this shape
int64_t attn_bwd_pe_part_rows(int64_t M, int64_t H, int64_t B, int64_t bsplit) {
  const int64_t nkb = (M + 255) / 256;
  const int slots = pe_bwd_slots((int)M, (int)H, bsplit);
  (void)B;
  return slots > 0 ? nkb + slots : nkb * bsplit;
}

static void attn_bwd_pe_impl(Tensor q, const Tensor* kv, Tensor dO, Tensor lse, Tensor delta, const Tensor* mean,
                             const Tensor* rstd, Tensor pix, Tensor dq, Tensor D, Tensor part, int64_t H, double scale,
                             bool accumulate, int64_t bsplit, const PeImplicit* impl, bool dq_zeroed = false,
                             bool d_zeroed = false) {
  for (const Tensor* t : {&q, &dO, &lse, &delta, &pix, &dq, &D, &part}) CHECK_CUDA(*t);
  const int C = (int)(H * 32);
  TORCH_CHECK(q.dim() == 3 && q.stride(2) == 1 && q.size(2) >= C, "q must be (B|1, Nq, >= C) with unit inner stride");
  const int Nq = (int)q.size(1);
  TORCH_CHECK(Nq >= 1 && Nq <= 32, "attn_bwd_pe: at most 32 queries");
  TORCH_CHECK(dO.dim() == 3 && dO.is_contiguous() && dO.size(1) == Nq && dO.size(2) == C, "dO must be (B, Nq, C)");
  const int B = (int)dO.size(0);
  TORCH_CHECK(q.size(0) == 1 || q.size(0) == B, "q batch must be 1 (broadcast) or B");
  const bool qb = q.size(0) == B && B > 1;
  int M;
  if (impl) {
    const Tensor& P = impl->P;
    CHECK_CUDA(P); CHECK_DT(P, torch::kBFloat16);
    M = (int)impl->pes.numel();
    TORCH_CHECK(P.dim() == 2 && P.is_contiguous() && P.size(1) == 2 * C && P.size(0) >= M && M > 0,
                "P must be (>= M, 2C) contiguous, M = pes.numel()");
    for (const Tensor* t : {&impl->pes, &impl->pesq, &impl->wt}) {
      CHECK_CUDA(*t); CHECK_DT(*t, torch::kFloat32);
      TORCH_CHECK(t->is_contiguous(), "attn_bwd_pe: contiguous PE operands");
    }
    TORCH_CHECK(impl->pes.numel() == M && impl->pesq.numel() == M && impl->wt.numel() == 6 * 2 * C,
                "attn_bwd_pe: pes / pesq (M), wt (6, 2C)");
    TORCH_CHECK(reinterpret_cast<uintptr_t>(P.data_ptr()) % 16 == 0 && reinterpret_cast<uintptr_t>(impl->wt.data_ptr()) % 16 == 0,
                "attn_bwd_pe: 16-byte aligned P / wt");
  } else {
    CHECK_CUDA(*kv);
    TORCH_CHECK(kv->dim() == 2 && kv->stride(1) == 1 && kv->size(1) >= 2 * C && kv->size(0) % B == 0,
                "kv must be (B*M, >= 2C) rows");
    M = (int)(kv->size(0) / B);
    TORCH_CHECK(kv->stride(0) % 8 == 0 && reinterpret_cast<uintptr_t>(kv->data_ptr()) % 16 == 0,
                "attn_bwd_pe: 16-byte aligned kv rows");
    TORCH_CHECK(mean->numel() == (int64_t)B * M && rstd->numel() == (int64_t)B * M && mean->is_contiguous() &&
                    rstd->is_contiguous(), "row statistics must be (B*M)");
    CHECK_DT(*mean, torch::kFloat32); CHECK_DT(*rstd, torch::kFloat32);
  }
  TORCH_CHECK(q.stride(1) % 8 == 0 && (!qb || q.stride(0) % 8 == 0) && reinterpret_cast<uintptr_t>(q.data_ptr()) % 16 == 0,
              "attn_bwd_pe: 16-byte aligned q rows");
  TORCH_CHECK(pix.dim() == 2 && pix.is_contiguous() && pix.size(0) == (int64_t)B * M && pix.size(1) >= 1 && pix.size(1) <= 4,
              "pix must be (B*M, nc <= 4)");
  const int nc = (int)pix.size(1);
  TORCH_CHECK(lse.is_contiguous() && delta.is_contiguous() && lse.numel() == (int64_t)B * Nq * H && delta.numel() == lse.numel(),
              "lse / delta must be (B, Nq, H)");
  TORCH_CHECK(dq.is_contiguous() && dq.numel() == (int64_t)(qb ? B : 1) * Nq * C,
              "dq must be (Nq, C) for broadcast queries (Σ over the batch), else (B, Nq, C)");
  TORCH_CHECK(D.is_contiguous() && D.size(0) == M && D.size(1) == 2 * C, "D must be (M, 2C) contiguous");
  const int nkb = (M + 255) / 256;
  TORCH_CHECK(bsplit >= 1 && bsplit <= B, "bsplit in [1, B]");
  const int slots = pe_bwd_slots(M, (int)H, bsplit);
  const int64_t prows = slots > 0 ? nkb + slots : (int64_t)nkb * bsplit;
  TORCH_CHECK(part.is_contiguous() && part.size(0) == prows && part.size(1) == (int64_t)(2 + nc) * 2 * C,
              "part must be (attn_bwd_pe_part_rows(M, H, B, bsplit), (2+nc)*2C)");
  for (const Tensor* t : {&lse, &delta, &pix, &dq, &D, &part}) CHECK_DT(*t, torch::kFloat32);
  TORCH_CHECK(!(g_det && bsplit > 1), "deterministic mode: attn_bwd_pe needs bsplit = 1");
  Tensor dq_part;
  if (g_det) dq_part = torch::empty({nkb, dq.numel()}, dq.options());
  else if (!dq_zeroed) dq.zero_();  // dq_zeroed: cleared by the preceding kernel's zero span
  pio::PeBwdArgs a{};
  a.q = bfp(q); a.q_bs = qb ? q.stride(0) : 0; a.q_rs = (int)q.stride(1);
  if (impl) {
    a.P = bfp(impl->P); a.pes = f32p(impl->pes); a.pesq = f32p(impl->pesq); a.wt = f32p(impl->wt);
    a.inv_k = (float)(1.0 / impl->kin); a.eps = (float)impl->eps;
  } else {
    a.kv = bfp(*kv); a.kv_rs = (int)kv->stride(0); a.mean = f32p(*mean); a.rstd = f32p(*rstd);
  }
  a.dO = bfp(dO); a.lse = f32p(lse); a.delta = f32p(delta); a.pix = f32p(pix);
  a.dq = g_det ? dq_part.data_ptr<float>() : dq.data_ptr<float>();
  a.dq_kbs = g_det ? dq.numel() : 0;
  a.D = D.data_ptr<float>(); a.part = part.data_ptr<float>();
  a.B = B; a.H = (int)H; a.Nq = Nq; a.M = M; a.C = C; a.nc = nc;
  a.scale = (float)scale; a.scale_log2 = (float)(scale * 1.4426950408889634);
  a.accumulate = accumulate ? 1 : 0;
  // the split batch groups add into D atomically; d_zeroed: cleared by the preceding kernel's zero span
  if (bsplit > 1 && !accumulate && !d_zeroed) D.zero_();
  Tensor dside, spair;
  if (slots > 0) {
    dside = torch::empty({slots, 256, 64}, D.options());
    spair = torch::empty({slots}, D.options().dtype(torch::kInt32));
    a.nbg = 4; a.nslots = slots; a.Dside = dside.data_ptr<float>(); a.side_pair = spair.data_ptr<int>();
    // slot rows (a side run writes only its head's columns) are cleared by the kernel itself
  }
  pio::attn_bwd_pe_launch(a, nkb, (int)bsplit, stream());
  if (g_det) dq.view({-1}).copy_(dq_part.sum(0));
}

void attn_bwd_pe(Tensor q, Tensor kv, Tensor dO, Tensor lse, Tensor delta, Tensor mean, Tensor rstd, Tensor pix,
                 Tensor dq, Tensor D, Tensor part, int64_t H, double scale, bool accumulate, int64_t bsplit,
                 bool dq_zeroed, bool d_zeroed) {
  attn_bwd_pe_impl(q, &kv, dO, lse, delta, &mean, &rstd, pix, dq, D, part, H, scale, accumulate, bsplit, nullptr,
                   dq_zeroed, d_zeroed);
}

// the same over implicit K/V (attention_pe.hip pe_kv_elem): no (B·M, 2C) K/V tensor, no row statistics
void attn_bwd_pe_implicit(Tensor q, Tensor P, Tensor pes, Tensor pesq, Tensor wt, Tensor dO, Tensor lse, Tensor delta,
                          Tensor pix, Tensor dq, Tensor D, Tensor part, int64_t H, double scale, int64_t kin, double eps,
                          bool accumulate, int64_t bsplit, bool dq_zeroed, bool d_zeroed) {
  PeImplicit im{P, pes, pesq, wt, (double)kin, eps};
  attn_bwd_pe_impl(q, nullptr, dO, lse, delta, nullptr, nullptr, pix, dq, D, part, H, scale, accumulate, bsplit, &im,
                   dq_zeroed, d_zeroed);
}

// encoder cross-attention forward over implicit K/V (attention_pe.hip attn_fwd_pe_kernel): queries
// (1 | B, Nq ≤ 32, ≥ C) bf16, head dim 32, no mask, no dropout; P' (M, 2C) bf16, pix (B·M, nc ≤ 4),
// pes / pesq (M), wt (6, 2C) → O (B, Nq, C) bf16, LSE (B, Nq, H) log2 units.  nsplit key splits.
std::vector<Tensor> attn_fwd_pe(Tensor q, Tensor P, Tensor pix, Tensor pes, Tensor pesq, Tensor wt, int64_t H,
                                double scale, int64_t kin, double eps, int64_t nsplit) {
  for (const Tensor* t : {&q, &P, &pix, &pes, &pesq, &wt}) CHECK_CUDA(*t);
  CHECK_DT(q, torch::kBFloat16); CHECK_DT(P, torch::kBFloat16);
  for (const Tensor* t : {&pix, &pes, &pesq, &wt}) {
    CHECK_DT(*t, torch::kFloat32);
    TORCH_CHECK(t->is_contiguous(), "attn_fwd_pe: contiguous fp32 operands");
  }
  const int C = (int)(H * 32);
  TORCH_CHECK(q.dim() == 3 && q.stride(2) == 1 && q.size(2) >= C && q.stride(1) % 8 == 0 &&
                  reinterpret_cast<uintptr_t>(q.data_ptr()) % 16 == 0, "q must be (B|1, Nq, >= C), 16-byte aligned rows");
  const int Nq = (int)q.size(1);
  TORCH_CHECK(Nq >= 1 && Nq <= 32, "attn_fwd_pe: at most 32 queries");
  const int M = (int)pes.numel();
  TORCH_CHECK(M > 0 && P.dim() == 2 && P.is_contiguous() && P.size(1) == 2 * C && P.size(0) >= M + 64 &&
                  reinterpret_cast<uintptr_t>(P.data_ptr()) % 16 == 0,
              "P must be (M + >= 64 zero pad rows, 2C) contiguous (pe_gemm pad_rows), M = pes.numel()");
  TORCH_CHECK(pix.dim() == 2 && pix.size(0) % M == 0 && pix.size(1) >= 1 && pix.size(1) <= 4, "pix must be (B*M, nc <= 4)");
  const int B = (int)(pix.size(0) / M);
  TORCH_CHECK(q.size(0) == 1 || q.size(0) == B, "q batch must be 1 (broadcast) or B");
  TORCH_CHECK(q.size(0) == 1 || q.stride(0) % 8 == 0, "q batch stride");
  TORCH_CHECK(pesq.numel() == M && wt.numel() == 6 * 2 * C &&
                  reinterpret_cast<uintptr_t>(wt.data_ptr()) % 16 == 0, "attn_fwd_pe: pes / pesq (M), wt (6, 2C)");
  if (nsplit <= 0) {  // one round of waves at the kernel's occupancy on this device
    int dev = 0, ncu = 256;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
    nsplit = pio::attn_fwd_pe_auto_splits(B, (int)H, ncu);
  }
  const int ns = (int)std::max<int64_t>(1, std::min<int64_t>(nsplit, (M + 31) / 32));
  auto o = torch::empty({B, Nq, C}, q.options());
  auto lse = torch::empty({B, Nq, H}, pix.options());
  auto Opart = torch::empty({(int64_t)ns * B * Nq * H * 32}, pix.options());
  auto MLpart = torch::empty({(int64_t)ns * B * Nq * H * 2}, pix.options());
  pio::PeFwdArgs a{};
  a.q = bfp(q); a.q_bs = q.size(0) == 1 ? 0 : q.stride(0); a.q_rs = (int)q.stride(1);
  a.P = bfp(P); a.pix = f32p(pix); a.pes = f32p(pes); a.pesq = f32p(pesq); a.wt = f32p(wt);
  a.Opart = Opart.data_ptr<float>(); a.MLpart = MLpart.data_ptr<float>();
  a.B = B; a.H = (int)H; a.Nq = Nq; a.M = M; a.C = C; a.nc = (int)pix.size(1); a.nsplit = ns;
  a.scale_log2 = (float)(scale * 1.4426950408889634); a.inv_k = (float)(1.0 / (double)kin); a.eps = (float)eps;
  pio::attn_fwd_pe_launch(a, stream());
  pio::attn_combine_launch(a.Opart, a.MLpart, bfp_mut(o), lse.data_ptr<float>(), ns, (long long)B * Nq * H, 32, stream());
  return {o, lse};
}

void set_deterministic(bool on) { g_det = on; }
bool get_deterministic() { return g_det; }

PYBIND11_MODULE(TORCH_EXTENSION_NAME, m) {
  TORCH_CHECK(pio::abi_struct_size(0) == (int)sizeof(pio::DropCfg) &&
                  pio::abi_struct_size(1) == (int)sizeof(pio::PostAttnGrads) &&
                  pio::abi_struct_size(2) == (int)sizeof(pio::SlabJob) &&
                  pio::abi_struct_size(3) == (int)sizeof(pio::AttnArgs),
              "perceiver_io_amd: binding.cpp struct mirrors disagree with the kernels (csrc/common.h, attention.hip)");
  m.def("set_deterministic", &set_deterministic);
  m.def("check_errors", &check_errors, py::arg("reset") = true);
  m.def("checked_build", &checked_build);
  m.def("get_deterministic", &get_deterministic);
  m.doc() = "Perceiver IO CDNA4 (gfx950) kernels";
  m.def("attn_fwd", &attn_fwd, py::arg("q"), py::arg("k"), py::arg("v"), py::arg("kmask"), py::arg("H"), py::arg("D"),
        py::arg("scale"), py::arg("dropout_p"), py::arg("seed"), py::arg("nsplit"), py::arg("site") = 0);
  m.def("attn_bwd", &attn_bwd, py::arg("q"), py::arg("k"), py::arg("v"), py::arg("kmask"), py::arg("o"), py::arg("dO"),
        py::arg("lse"), py::arg("delta_in"), py::arg("H"), py::arg("D"), py::arg("scale"), py::arg("dropout_p"),
        py::arg("seed"), py::arg("dq_out"), py::arg("dk_out"), py::arg("dv_out"), py::arg("kv_accumulate") = false,
        py::arg("site") = 0, py::arg("dq_zeroed") = false, py::arg("kv_zeroed") = false,
        py::arg("job_slab") = py::none(), py::arg("job_dsts") = std::vector<Tensor>{},
        py::arg("job_offs") = std::vector<int64_t>{});
  m.def("attn_bwd_zero_plan", &pio::attn_bwd_zero_plan, py::arg("B"), py::arg("H"), py::arg("Nq"), py::arg("Nk"),
        py::arg("D"));
  m.def("ln_linear_fwd", &ln_linear_fwd, py::arg("x"), py::arg("lnw"), py::arg("lnb"), py::arg("eps"), py::arg("w"),
        py::arg("bias"), py::arg("act"), py::arg("res"), py::arg("out_bf16"), py::arg("save_stats"),
        py::arg("pe") = py::none(), py::arg("kin") = -1, py::arg("pe_index") = py::none());
  m.def("post_attn_fwd", &post_attn_fwd, py::arg("o"), py::arg("x"), py::arg("wo"), py::arg("bo"), py::arg("g2"),
        py::arg("be2"), py::arg("eps"), py::arg("w1"), py::arg("b1"), py::arg("w2"), py::arg("b2"),
        py::arg("seed") = py::none(), py::arg("site") = 0, py::arg("p") = 0.0);
  m.def("sa_layer_fwd", &sa_layer_fwd, py::arg("qkv"), py::arg("x"), py::arg("N"), py::arg("scale"), py::arg("wo"),
        py::arg("bo"), py::arg("g2"), py::arg("be2"), py::arg("eps"), py::arg("w1"), py::arg("b1"), py::arg("w2"),
        py::arg("b2"), py::arg("lnw") = py::none(), py::arg("lnb") = py::none(), py::arg("wq") = py::none(),
        py::arg("bq") = py::none(), py::arg("seed") = py::none(), py::arg("site") = 0, py::arg("p") = 0.0);
  m.def("sb_fwd", &sb_fwd, py::arg("x"), py::arg("params"), py::arg("scale"), py::arg("eps"),
        py::arg("pre") = std::vector<Tensor>{}, py::arg("post") = std::vector<Tensor>{});
  m.def("sb_bwd", &sb_bwd, py::arg("dz"), py::arg("x0"), py::arg("saved"), py::arg("params"),
        py::arg("scale"), py::arg("eps"), py::arg("pre") = std::vector<Tensor>{},
        py::arg("pre_saved") = std::vector<Tensor>{}, py::arg("zero_out") = py::none(),
        py::arg("post") = std::vector<Tensor>{}, py::arg("post_io") = std::vector<Tensor>{});
  m.def("sb_wgrad", &sb_wgrad, py::arg("jobs"), py::arg("job_slab") = py::none(),
        py::arg("job_dsts") = std::vector<Tensor>(), py::arg("job_offs") = std::vector<int64_t>());
  m.def("post_attn_ln_linear_fwd", &post_attn_ln_linear_fwd, py::arg("o"), py::arg("x"), py::arg("wo"), py::arg("bo"),
        py::arg("g2"), py::arg("be2"), py::arg("eps"), py::arg("w1"), py::arg("b1"), py::arg("w2"), py::arg("b2"),
        py::arg("lnw"), py::arg("lnb"), py::arg("wq"), py::arg("bq"), py::arg("seed") = py::none(),
        py::arg("site") = 0, py::arg("p") = 0.0);
  m.def("ln_linear_post_attn_bwd", &ln_linear_post_attn_bwd, py::arg("g"), py::arg("wq"), py::arg("x"),
        py::arg("mean1"), py::arg("rstd1"), py::arg("lnw"), py::arg("lnb"), py::arg("dres"), py::arg("ll_grads"),
        py::arg("y"), py::arg("m2"), py::arg("r2"), py::arg("u"), py::arg("o"), py::arg("wo"), py::arg("w1"),
        py::arg("w2"), py::arg("g2"), py::arg("be2"), py::arg("H"), py::arg("pa_grads"),
        py::arg("job_slab") = py::none(), py::arg("job_dsts") = std::vector<Tensor>(),
        py::arg("job_offs") = std::vector<int64_t>(), py::arg("seed") = py::none(), py::arg("site") = 0,
        py::arg("p") = 0.0, py::arg("zero_out") = py::none(), py::arg("att_qkv") = py::none(),
        py::arg("att_lse") = py::none(), py::arg("att_out") = py::none(), py::arg("att_scale") = 0.0);
  m.def("post_attn_bwd", &post_attn_bwd, py::arg("dz"), py::arg("y"), py::arg("m2"), py::arg("r2"), py::arg("u"),
        py::arg("o"), py::arg("wo"), py::arg("w1"), py::arg("w2"), py::arg("g2"), py::arg("be2"), py::arg("H"),
        py::arg("grads"), py::arg("slab") = false, py::arg("job_slab") = py::none(),
        py::arg("job_dsts") = std::vector<Tensor>(), py::arg("job_offs") = std::vector<int64_t>(),
        py::arg("seed") = py::none(), py::arg("site") = 0, py::arg("p") = 0.0, py::arg("zero_out") = py::none());
  m.def("ln_linear_bwd", &ln_linear_bwd, py::arg("g"), py::arg("w"), py::arg("x"), py::arg("mean"), py::arg("rstd"),
        py::arg("lnw"), py::arg("lnb"), py::arg("dres"), py::arg("need_dx"), py::arg("dlnw"), py::arg("dlnb"),
        py::arg("dW"), py::arg("db"), py::arg("pe") = py::none(), py::arg("kin") = -1, py::arg("slab") = false,
        py::arg("job_slab") = py::none(), py::arg("job_dsts") = std::vector<Tensor>(),
        py::arg("job_offs") = std::vector<int64_t>(), py::arg("dx_out") = py::none(), py::arg("pe_index") = py::none());
  m.def("wgrad", &wgrad, py::arg("g"), py::arg("a"), py::arg("amode"), py::arg("mean"), py::arg("rstd"), py::arg("lnw"),
        py::arg("lnb"), py::arg("rows_per_wg"), py::arg("dW"), py::arg("db"), py::arg("pe") = py::none(),
        py::arg("kin") = -1, py::arg("pe_index") = py::none());
  m.def("mlm_select", &mlm_select, py::arg("labels"), py::arg("cap"), py::arg("gcap"), py::arg("sticky") = py::none(),
        py::arg("queries") = py::none());
  m.def("index_add_rows", &index_add_rows);
  m.def("gather_rows", &gather_rows, py::arg("src"), py::arg("idx"));
  m.def("batch_sum2", &batch_sum2, py::arg("a"), py::arg("b"), py::arg("ob_acc") = py::none());
  m.def("pixel_ce_fwd", &pixel_ce_fwd);
  m.def("pixel_ce_bwd", &pixel_ce_bwd);
  m.def("stage_step", &stage_step, py::arg("dsts"), py::arg("srcs"), py::arg("hyper_dst") = py::none(),
        py::arg("hyper") = std::vector<double>{}, py::arg("seed_dst") = py::none(),
        py::arg("seeds") = std::vector<int64_t>{});
  m.def("ce_fwd", &ce_fwd, py::arg("h"), py::arg("idx"), py::arg("labels"), py::arg("w"), py::arg("bias"),
        py::arg("count"), py::arg("zero_out") = py::none(), py::arg("count_labels") = false);
  m.def("ce_bwd", &ce_bwd, py::arg("h"), py::arg("labels"), py::arg("w"), py::arg("bias"),
        py::arg("lse"), py::arg("gout"), py::arg("count"), py::arg("dH"), py::arg("dW"), py::arg("db"),
        py::arg("accumulate"), py::arg("rowmap") = py::none(), py::arg("slab") = false, py::arg("u") = py::none(),
        py::arg("u_ml") = py::none());
  m.def("embed_fwd", &embed_fwd);
  m.def("embed_bwd", &embed_bwd, py::arg("ids"), py::arg("g"), py::arg("dE"), py::arg("dP"), py::arg("scale"),
        py::arg("job_slab") = py::none(), py::arg("job_dsts") = std::vector<Tensor>(),
        py::arg("job_offs") = std::vector<int64_t>());
  m.def("text_mask", &text_mask, py::arg("x"), py::arg("pad"), py::arg("state"), py::arg("unk"), py::arg("mask"),
        py::arg("p"), py::arg("lo"), py::arg("hi"), py::arg("advance") = true);
  m.def("sumsq", &sumsq);
  m.def("adamw", &adamw, py::arg("p"), py::arg("g"), py::arg("m"), py::arg("v"), py::arg("shadow"), py::arg("hyper"),
        py::arg("eps"), py::arg("wd"), py::arg("clip"), py::arg("gscale"), py::arg("l2") = false,
        py::arg("zero_grad") = false, py::arg("loss_src") = py::none(), py::arg("loss_ring") = py::none(),
        py::arg("norm_part") = py::none());
  m.def("cast_bf16", &cast_bf16);
  m.def("reduce_probe", &reduce_probe);
  m.def("fold_replicas", &fold_replicas);
  m.def("slab_reduce", &slab_reduce);
  m.def("pe_proj_fwd", &pe_proj_fwd);
  m.def("pe_gemm", &pe_gemm, py::arg("A"), py::arg("B"), py::arg("bf16_out") = false, py::arg("pad_rows") = 0);
  m.def("attn_fwd_pe", &attn_fwd_pe);
  m.def("sa_block_fwd", &sa_block_fwd, py::arg("qkv0"), py::arg("x0"), py::arg("N"), py::arg("scale"), py::arg("eps"),
        py::arg("wo"), py::arg("bo"), py::arg("g2"), py::arg("be2"), py::arg("w1"), py::arg("b1"), py::arg("w2"),
        py::arg("b2"), py::arg("lnw"), py::arg("lnb"), py::arg("wq"), py::arg("bq"), py::arg("seed") = py::none(),
        py::arg("p") = 0.0);
  m.def("persist_errors", &persist_errors, py::arg("reset") = true);
  m.def("persist_set_spin_limit", [](int64_t n) { pio::persist_set_spin_limit((unsigned)n); }, py::arg("n"));
  m.def("attn_bwd_pe_part_rows", &attn_bwd_pe_part_rows);
  m.def("attn_bwd_pe_implicit", &attn_bwd_pe_implicit, py::arg("q"), py::arg("P"), py::arg("pes"), py::arg("pesq"),
        py::arg("wt"), py::arg("dO"), py::arg("lse"), py::arg("delta"), py::arg("pix"), py::arg("dq"), py::arg("D"),
        py::arg("part"), py::arg("H"), py::arg("scale"), py::arg("kin"), py::arg("eps"), py::arg("accumulate"),
        py::arg("bsplit"), py::arg("dq_zeroed") = false, py::arg("d_zeroed") = false);
  m.def("pe_weight_prep", &pe_weight_prep, py::arg("W"), py::arg("g"), py::arg("b"), py::arg("bias"), py::arg("nc"),
        py::arg("Kp"), py::arg("W2") = py::none());
  m.def("pe_grads", &pe_grads);
  m.def("pe_proj_bwd", &pe_proj_bwd);
  m.def("attn_bwd_pe", &attn_bwd_pe, py::arg("q"), py::arg("kv"), py::arg("dO"), py::arg("lse"), py::arg("delta"),
        py::arg("mean"), py::arg("rstd"), py::arg("pix"), py::arg("dq"), py::arg("D"), py::arg("part"), py::arg("H"),
        py::arg("scale"), py::arg("accumulate"), py::arg("bsplit"), py::arg("dq_zeroed") = false,
        py::arg("d_zeroed") = false);
  m.attr("arch") = "gfx950";
}
