// Argument block shared by the short-sequence attention kernels
// (attn_small.hip: scalar fallback; attn_mfma.hip: MFMA path for S <= 16).
#pragma once
#include <cstdint>

#include <hip/hip_runtime.h>

namespace ccmpi {
namespace dev {
namespace attn {

struct AttnArgs {
  const uint16_t* qkv;  // [B*S][ld_qkv]
  uint16_t* o;          // [B*S][ld_o]
  float* lse;           // [B*Hl][S]
  const uint16_t* dout; // [B*S][ld_o]   (bwd)
  uint16_t* dqkv;       // [B*S][ld_qkv] (bwd)
  float* dbias;         // [3*Hl*D] fp32, += column sums of dqkv (bwd, optional)
  int B, S, Hl, D, ld_qkv, ld_o;
  float scale;
  uint16_t* pool;       // fwd, optional: [B][ld_pool] bf16 mean over the S rows of O
  int ld_pool;
  int dout_bstride;     // bwd: dO row (b, i) at dout + b*dout_bstride + i*dout_rstride + h*D
  int dout_rstride;     //      (rstride 0 = the pooled-gradient broadcast over the S rows)
  // Pooled row-parallel fc_o fused into the MFMA kernels (optional; Hl must divide
  // the 4 waves of a workgroup, n_out <= 16).  W_o is [n_out][ld_wo] bf16 whose
  // columns are this rank's attention features (h*D + d).
  const uint16_t* wo;
  int ld_wo, n_out;
  float* zp;            // fwd: zp[b][0..n_out) = pool[b] . W_o^T (+ bo), fp32, row stride ld_zp
  int ld_zp;
  const float* bo;      // fwd: optional output bias [n_out]
  const uint16_t* dz;   // bwd: dO rows of sequence b = dz_scale * (dz[b] . W_o), broadcast over the S
  int ld_dz;            //      rows (replaces dout; dz is [B][ld_dz] bf16)
  float dz_scale;
  // Per-token row-parallel fc_o fused into the MFMA forward (the reference layer's shape,
  // model/func_impl.py:94-109: every token's partial output, not the pooled one):
  // z[b*S + i][0..16) = bf16(O[b, i]) . W_o^T (+ bo), the Hl local heads summed in head order,
  // fp32 rows of ld_zt floats.  zrows == 0: into ztok (local).  zrows > 0 (push): row block j
  // = rows [j zrows, (j+1) zrows) goes to zpush[j] (rank j's inbox slot for this rank, peer-
  // mapped), stored write-through; DeviceComm::inbox_to_local then completes the TP sum.
  float* ztok;
  int ld_zt;
  int zrows;
  float* zpush[16];
  // Fused QKV projection (k_qkv_attn16_fwd, the harness forward): qkv = X W^T + b computed in
  // the attention kernel from the patch rows X ([B*S][ld_xq] bf16, kq <= 80 columns) and the
  // folded weight W ([3 Hl D][ld_wq] bf16: q rows, then k, then v) with the fp32 bias bq;
  // qkv_out (optional, [B*S][ld_qkv] bf16): the projection is also stored, for a backward
  const uint16_t* xq;
  int ld_xq, kq;
  const uint16_t* wq;
  int ld_wq;
  const float* bq;
  uint16_t* qkv_out;
  // img (optional, [B][28 * 28] fp32 MNIST images): the kernel builds X itself (7 x 7 patch
  // pixels, a 1, the one-hot position -- k_patchify's rows, bitwise) and, with xq_out, stores
  // them ([B*S][ld_xq] bf16) for the backward; xq is then unused
  const float* img;
  uint16_t* xq_out;
  // fused QKV in image mode, optional: the NEXT forward's weight fold fold_out = bf16(fold_wq .
  // fold_we) ([fold_R][fold_kp] from fp32 [fold_R][fold_d] and [fold_d][fold_kp]), computed by
  // the workgroups once their attention work is done -- bitwise the fold_emb_qkv MFMA
  // kernel's result (same per-slice MFMA chains, same summation order)
  const float* fold_wq;
  int ld_fold_wq;
  const float* fold_we;
  int ld_fold_we;
  uint16_t* fold_out;
  int ld_fold_out, fold_R, fold_d, fold_kp;
  int fold_at_start;  // 1: the fold runs before the attention work (its loads under W_h's), 0: after
  // set by launch_qkv_fwd_mfma: 0 = every workgroup takes its pair blocks grid-stride; k + 1 = the
  // fold-owning workgroups stop after k rounds and the others share the remaining blocks
  int fold_sched;
  // diagnostic (fused QKV forward): per wave kTStamps shader-clock stamps of the kernel's
  // phases ([grid * 4 waves][32] u64; s_memtime, buffered in LDS, stored at the end), or null
  unsigned long long* tstamp;
};
constexpr int kTStamps = 32;

// MFMA path (attn_mfma.hip): S <= 16, D in {32, 64, 128}, 16-B aligned rows.
bool mfma_supported(const AttnArgs& a, bool bwd);
void launch_fwd_mfma(const AttnArgs& a, hipStream_t stream);
void launch_bwd_mfma(const AttnArgs& a, hipStream_t stream);
void launch_qkv_fwd_mfma(const AttnArgs& a, hipStream_t stream);  // fused QKV + attention + token fc_o
extern int g_qkv_grid_cap;  // workgroups of the fused QKV forward (persistent grid)
extern int g_qkv_fold_sched;  // fold-aware block schedule of the fused forward: -1 env, 0 off, 1 on
extern int g_qkv_fold_grid;   // ... and its grid widened by the fold's tiles at small batches (1) or not (0)
extern int g_bwd_grid_cap;  // workgroups of the backward kernel when it also reduces the bias gradient

}  // namespace attn
}  // namespace dev
}  // namespace ccmpi
