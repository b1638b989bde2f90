// FlashAttention forward prototype: 8-wave ping-pong (two half-workgroups one segment apart),
// 3-deep K/V LDS-DMA rings.  Derived from the DSL kernel of example_mha_fwd_pipelined.py
// (b1 h64 s4096 d128, block 256x64, 512 threads); same signature, grid and block, so
// scripts/proto/fa_pp_ab.py swaps it in through the postproc hook.
//   PP=1: waves 4-7 run one barrier behind waves 0-3: while one half issues the MFMAs of
//   S(t) = Q K(t)^T and O += P(t-1) V(t-1), its SIMD partner runs softmax(t-1) (VALU/exp).
//   PP=0: same body, all waves in lockstep (two barriers per tile).
#include "tl/tl.h"
#ifndef PP
#define PP 1
#endif
#ifndef PRIO
#define PRIO 0
#endif
#define NST 3
#define NT (SEQ / 64)
#ifndef NOPIN
#define BAR() do { __builtin_amdgcn_sched_barrier(0); tl::barrier_raw(); __builtin_amdgcn_sched_barrier(0); } while (0)
#else
#define BAR() tl::barrier_raw()
#endif

extern "C" __global__ void __launch_bounds__(512) flashattn_pipelined_kernel(bfloat16_t* __restrict__ Q, bfloat16_t* __restrict__ K, bfloat16_t* __restrict__ V, bfloat16_t* __restrict__ Output) {
  __shared__ __attribute__((aligned(1024))) char tl_smem[NST * 32768];
  const int tid_ = threadIdx.x;
  const int lane_ = tid_ & 63;
  const int wave_ = __builtin_amdgcn_readfirstlane(tid_ >> 6);
  const int bx = blockIdx.x;
  const int by = blockIdx.y;
  const int bz = blockIdx.z;
  bfloat16_t* K_ring = reinterpret_cast<bfloat16_t*>(tl_smem);
  bfloat16_t* V_ring = reinterpret_cast<bfloat16_t*>(tl_smem + NST * 16384);
  bfloat16_t vtmp0[8];
  bfloat16_t vtmp1[8];
  bfloat16_t vtmp2[8];
  bfloat16_t vtmp3[8];
  bfloat16_t vtmp4[8];
  bfloat16_t vtmp5[8];
  bfloat16_t vtmp6[8];
  bfloat16_t vtmp7[8];
  bfloat16_t Q_s[64];
  tl::load_vec<bfloat16_t, 8>(*reinterpret_cast<bfloat16_t(*)[8]>(&vtmp0[0]), &Q[((((bz * 33554432) + (((bx * 256) + (((((tid_ / 16) / 4) % 8) * 32) + (tid_ % 16))) * 8192)) + (by * 128)) + (((tid_ / 16) % 4) * 8))]);
  Q_s[0] = vtmp0[0];
  Q_s[1] = vtmp0[1];
  Q_s[2] = vtmp0[2];
  Q_s[3] = vtmp0[3];
  Q_s[4] = vtmp0[4];
  Q_s[5] = vtmp0[5];
  Q_s[6] = vtmp0[6];
  Q_s[7] = vtmp0[7];
  tl::load_vec<bfloat16_t, 8>(*reinterpret_cast<bfloat16_t(*)[8]>(&vtmp1[0]), &Q[((((bz * 33554432) + (((bx * 256) + (((((tid_ / 16) / 4) % 8) * 32) + (tid_ % 16))) * 8192)) + (by * 128)) + ((((tid_ / 16) % 4) * 8) + 32))]);
  Q_s[8] = vtmp1[0];
  Q_s[9] = vtmp1[1];
  Q_s[10] = vtmp1[2];
  Q_s[11] = vtmp1[3];
  Q_s[12] = vtmp1[4];
  Q_s[13] = vtmp1[5];
  Q_s[14] = vtmp1[6];
  Q_s[15] = vtmp1[7];
  tl::load_vec<bfloat16_t, 8>(*reinterpret_cast<bfloat16_t(*)[8]>(&vtmp2[0]), &Q[((((bz * 33554432) + (((bx * 256) + (((((tid_ / 16) / 4) % 8) * 32) + (tid_ % 16))) * 8192)) + (by * 128)) + ((((tid_ / 16) % 4) * 8) + 64))]);
  Q_s[16] = vtmp2[0];
  Q_s[17] = vtmp2[1];
  Q_s[18] = vtmp2[2];
  Q_s[19] = vtmp2[3];
  Q_s[20] = vtmp2[4];
  Q_s[21] = vtmp2[5];
  Q_s[22] = vtmp2[6];
  Q_s[23] = vtmp2[7];
  tl::load_vec<bfloat16_t, 8>(*reinterpret_cast<bfloat16_t(*)[8]>(&vtmp3[0]), &Q[((((bz * 33554432) + (((bx * 256) + (((((tid_ / 16) / 4) % 8) * 32) + (tid_ % 16))) * 8192)) + (by * 128)) + ((((tid_ / 16) % 4) * 8) + 96))]);
  Q_s[24] = vtmp3[0];
  Q_s[25] = vtmp3[1];
  Q_s[26] = vtmp3[2];
  Q_s[27] = vtmp3[3];
  Q_s[28] = vtmp3[4];
  Q_s[29] = vtmp3[5];
  Q_s[30] = vtmp3[6];
  Q_s[31] = vtmp3[7];
  tl::load_vec<bfloat16_t, 8>(*reinterpret_cast<bfloat16_t(*)[8]>(&vtmp4[0]), &Q[((((bz * 33554432) + (((bx * 256) + ((((((tid_ / 16) / 4) % 8) * 32) + (tid_ % 16)) + 16)) * 8192)) + (by * 128)) + (((tid_ / 16) % 4) * 8))]);
  Q_s[32] = vtmp4[0];
  Q_s[33] = vtmp4[1];
  Q_s[34] = vtmp4[2];
  Q_s[35] = vtmp4[3];
  Q_s[36] = vtmp4[4];
  Q_s[37] = vtmp4[5];
  Q_s[38] = vtmp4[6];
  Q_s[39] = vtmp4[7];
  tl::load_vec<bfloat16_t, 8>(*reinterpret_cast<bfloat16_t(*)[8]>(&vtmp5[0]), &Q[((((bz * 33554432) + (((bx * 256) + ((((((tid_ / 16) / 4) % 8) * 32) + (tid_ % 16)) + 16)) * 8192)) + (by * 128)) + ((((tid_ / 16) % 4) * 8) + 32))]);
  Q_s[40] = vtmp5[0];
  Q_s[41] = vtmp5[1];
  Q_s[42] = vtmp5[2];
  Q_s[43] = vtmp5[3];
  Q_s[44] = vtmp5[4];
  Q_s[45] = vtmp5[5];
  Q_s[46] = vtmp5[6];
  Q_s[47] = vtmp5[7];
  tl::load_vec<bfloat16_t, 8>(*reinterpret_cast<bfloat16_t(*)[8]>(&vtmp6[0]), &Q[((((bz * 33554432) + (((bx * 256) + ((((((tid_ / 16) / 4) % 8) * 32) + (tid_ % 16)) + 16)) * 8192)) + (by * 128)) + ((((tid_ / 16) % 4) * 8) + 64))]);
  Q_s[48] = vtmp6[0];
  Q_s[49] = vtmp6[1];
  Q_s[50] = vtmp6[2];
  Q_s[51] = vtmp6[3];
  Q_s[52] = vtmp6[4];
  Q_s[53] = vtmp6[5];
  Q_s[54] = vtmp6[6];
  Q_s[55] = vtmp6[7];
  tl::load_vec<bfloat16_t, 8>(*reinterpret_cast<bfloat16_t(*)[8]>(&vtmp7[0]), &Q[((((bz * 33554432) + (((bx * 256) + ((((((tid_ / 16) / 4) % 8) * 32) + (tid_ % 16)) + 16)) * 8192)) + (by * 128)) + ((((tid_ / 16) % 4) * 8) + 96))]);
  Q_s[56] = vtmp7[0];
  Q_s[57] = vtmp7[1];
  Q_s[58] = vtmp7[2];
  Q_s[59] = vtmp7[3];
  Q_s[60] = vtmp7[4];
  Q_s[61] = vtmp7[5];
  Q_s[62] = vtmp7[6];
  Q_s[63] = vtmp7[7];
  float acc_s[32];
  bfloat16_t acc_s_cast[32];
  float acc_o[64];
  float scores_max[2];
  float scores_max_prev[2];
  float scores_scale[2];
  float scores_sum[2];
  float logsum[2];
  int rescale[1];
#pragma unroll
  for (int i = 0; i < 64; ++i) acc_o[i] = 0.0f;
  logsum[0] = logsum[1] = 0.0f;
  scores_max[0] = scores_max[1] = (-1073741824.0f);
  scores_scale[0] = scores_scale[1] = 1.0f;
  rescale[0] = 0;
#if PRIO
  if (wave_ >= 4) __builtin_amdgcn_s_setprio(1);
#endif
  bfloat16_t* K_src1 = reinterpret_cast<bfloat16_t*>((&K[((((bz * 33554432) + ((((wave_ * 64) + lane_) / 16) * 8192)) + (by * 128)) + (((((wave_ * 64) + lane_) % 16) ^ (((((((wave_ * 64) + lane_) / 16) & 1) << 1) ^ ((((((wave_ * 64) + lane_) / 16) >> 1) & 1) << 2)) ^ ((((((wave_ * 64) + lane_) / 16) >> 2) & 1) << 3))) * 8))]));
  bfloat16_t* K_src2 = reinterpret_cast<bfloat16_t*>((&K[((((bz * 33554432) + (((((8 + wave_) * 64) + lane_) / 16) * 8192)) + (by * 128)) + ((((((8 + wave_) * 64) + lane_) % 16) ^ ((((((((8 + wave_) * 64) + lane_) / 16) & 1) << 1) ^ (((((((8 + wave_) * 64) + lane_) / 16) >> 1) & 1) << 2)) ^ (((((((8 + wave_) * 64) + lane_) / 16) >> 2) & 1) << 3))) * 8))]));
  bfloat16_t* V_src3 = reinterpret_cast<bfloat16_t*>((&V[((((bz * 33554432) + ((((wave_ * 64) + lane_) / 16) * 8192)) + (by * 128)) + (((((wave_ * 64) + lane_) % 16) ^ (((((((wave_ * 64) + lane_) / 16) & 1) << 1) ^ ((((((wave_ * 64) + lane_) / 16) >> 1) & 1) << 2)) ^ ((((((wave_ * 64) + lane_) / 16) >> 2) & 1) << 3))) * 8))]));
  bfloat16_t* V_src4 = reinterpret_cast<bfloat16_t*>((&V[((((bz * 33554432) + (((((8 + wave_) * 64) + lane_) / 16) * 8192)) + (by * 128)) + ((((((8 + wave_) * 64) + lane_) % 16) ^ ((((((((8 + wave_) * 64) + lane_) / 16) & 1) << 1) ^ (((((((8 + wave_) * 64) + lane_) / 16) >> 1) & 1) << 2)) ^ (((((((8 + wave_) * 64) + lane_) / 16) >> 2) & 1) << 3))) * 8))]));
#define ISSUE_K(t) do { const int s_ = (t) % NST; tl::glds16(&K_src1[(t) * 524288], &K_ring[s_ * 8192 + wave_ * 512]); tl::glds16(&K_src2[(t) * 524288], &K_ring[s_ * 8192 + (8 + wave_) * 512]); } while (0)
#define ISSUE_V(t) do { const int s_ = (t) % NST; tl::glds16(&V_src3[(t) * 524288], &V_ring[s_ * 8192 + wave_ * 512]); tl::glds16(&V_src4[(t) * 524288], &V_ring[s_ * 8192 + (8 + wave_) * 512]); } while (0)
#define S_GEMM(t) do { _Pragma("unroll") for (int i = 0; i < 32; ++i) acc_s[i] = 0.0f; \
    tl::gemm_rs<bfloat16_t, 256, 64, 128, 8, 1, true, 128, 12816u, 0>((&Q_s[0]), (&K_ring[((t) % NST) * 8192]), (&acc_s[0]), wave_); } while (0)
#define PV_GEMM(t) tl::gemm_rs<bfloat16_t, 256, 128, 64, 8, 1, false, 128, 12816u, 1>((&acc_s_cast[0]), (&V_ring[((t) % NST) * 8192]), (&acc_o[0]), wave_)
  ISSUE_K(0);
  ISSUE_V(0);
  ISSUE_K(1);
  tl::wait_vmcnt<4>();
  BAR();
  S_GEMM(0);
  tl::wait_vmcnt<0>();
  BAR();
#if PP
  if (wave_ >= 4) BAR();
#endif
  // softmax(0), then the tiles two (K) / one (V) ahead
    scores_max_prev[0] = scores_max[0];
    scores_max_prev[1] = scores_max[1];
    {
      const float red0_2 = __builtin_fmaxf(__builtin_fmaxf(__builtin_fmaxf(__builtin_fmaxf(acc_s[0], acc_s[1]), __builtin_fmaxf(acc_s[2], acc_s[3])), __builtin_fmaxf(__builtin_fmaxf(acc_s[4], acc_s[5]), __builtin_fmaxf(acc_s[6], acc_s[7]))), __builtin_fmaxf(__builtin_fmaxf(__builtin_fmaxf(acc_s[8], acc_s[9]), __builtin_fmaxf(acc_s[10], acc_s[11])), __builtin_fmaxf(__builtin_fmaxf(acc_s[12], acc_s[13]), __builtin_fmaxf(acc_s[14], acc_s[15]))));
      const float red1_2 = __builtin_fmaxf(__builtin_fmaxf(__builtin_fmaxf(__builtin_fmaxf(acc_s[16], acc_s[17]), __builtin_fmaxf(acc_s[18], acc_s[19])), __builtin_fmaxf(__builtin_fmaxf(acc_s[20], acc_s[21]), __builtin_fmaxf(acc_s[22], acc_s[23]))), __builtin_fmaxf(__builtin_fmaxf(__builtin_fmaxf(acc_s[24], acc_s[25]), __builtin_fmaxf(acc_s[26], acc_s[27])), __builtin_fmaxf(__builtin_fmaxf(acc_s[28], acc_s[29]), __builtin_fmaxf(acc_s[30], acc_s[31]))));
      const float redl0_2 = tl::lane_allreduce<tl::MaxOp, 48>(red0_2);
      const float redl1_2 = tl::lane_allreduce<tl::MaxOp, 48>(red1_2);
      scores_max_prev[0] = __builtin_fmaxf(scores_max_prev[0], redl0_2);
      scores_max_prev[1] = __builtin_fmaxf(scores_max_prev[1], redl1_2);
    }
    rescale[0] = 0;
    {
      if ((((scores_max_prev[0] - scores_max[0]) * 0.1275174307460247f) > 8.0f)) {
        scores_scale[0] = tl::fast_exp2(((scores_max[0] - scores_max_prev[0]) * 0.1275174307460247f));
        scores_max[0] = scores_max_prev[0];
        rescale[0] = 1;
      } else {
        scores_scale[0] = 1.0f;
      }
    }
    {
      if ((((scores_max_prev[1] - scores_max[1]) * 0.1275174307460247f) > 8.0f)) {
        scores_scale[1] = tl::fast_exp2(((scores_max[1] - scores_max_prev[1]) * 0.1275174307460247f));
        scores_max[1] = scores_max_prev[1];
        rescale[0] = 1;
      } else {
        scores_scale[1] = 1.0f;
      }
    }
    acc_s[0] = tl::fast_exp2(((acc_s[0] * 0.1275174307460247f) - (scores_max[0] * 0.1275174307460247f)));
    acc_s[1] = tl::fast_exp2(((acc_s[1] * 0.1275174307460247f) - (scores_max[0] * 0.1275174307460247f)));
    acc_s[2] = tl::fast_exp2(((acc_s[2] * 0.1275174307460247f) - (scores_max[0] * 0.1275174307460247f)));
    acc_s[3] = tl::fast_exp2(((acc_s[3] * 0.1275174307460247f) - (scores_max[0] * 0.1275174307460247f)));
    acc_s[4] = tl::fast_exp2(((acc_s[4] * 0.1275174307460247f) - (scores_max[0] * 0.1275174307460247f)));
    acc_s[5] = tl::fast_exp2(((acc_s[5] * 0.1275174307460247f) - (scores_max[0] * 0.1275174307460247f)));
    acc_s[6] = tl::fast_exp2(((acc_s[6] * 0.1275174307460247f) - (scores_max[0] * 0.1275174307460247f)));
    acc_s[7] = tl::fast_exp2(((acc_s[7] * 0.1275174307460247f) - (scores_max[0] * 0.1275174307460247f)));
    acc_s[8] = tl::fast_exp2(((acc_s[8] * 0.1275174307460247f) - (scores_max[0] * 0.1275174307460247f)));
    acc_s[9] = tl::fast_exp2(((acc_s[9] * 0.1275174307460247f) - (scores_max[0] * 0.1275174307460247f)));
    acc_s[10] = tl::fast_exp2(((acc_s[10] * 0.1275174307460247f) - (scores_max[0] * 0.1275174307460247f)));
    acc_s[11] = tl::fast_exp2(((acc_s[11] * 0.1275174307460247f) - (scores_max[0] * 0.1275174307460247f)));
    acc_s[12] = tl::fast_exp2(((acc_s[12] * 0.1275174307460247f) - (scores_max[0] * 0.1275174307460247f)));
    acc_s[13] = tl::fast_exp2(((acc_s[13] * 0.1275174307460247f) - (scores_max[0] * 0.1275174307460247f)));
    acc_s[14] = tl::fast_exp2(((acc_s[14] * 0.1275174307460247f) - (scores_max[0] * 0.1275174307460247f)));
    acc_s[15] = tl::fast_exp2(((acc_s[15] * 0.1275174307460247f) - (scores_max[0] * 0.1275174307460247f)));
    acc_s[16] = tl::fast_exp2(((acc_s[16] * 0.1275174307460247f) - (scores_max[1] * 0.1275174307460247f)));
    acc_s[17] = tl::fast_exp2(((acc_s[17] * 0.1275174307460247f) - (scores_max[1] * 0.1275174307460247f)));
    acc_s[18] = tl::fast_exp2(((acc_s[18] * 0.1275174307460247f) - (scores_max[1] * 0.1275174307460247f)));
    acc_s[19] = tl::fast_exp2(((acc_s[19] * 0.1275174307460247f) - (scores_max[1] * 0.1275174307460247f)));
    acc_s[20] = tl::fast_exp2(((acc_s[20] * 0.1275174307460247f) - (scores_max[1] * 0.1275174307460247f)));
    acc_s[21] = tl::fast_exp2(((acc_s[21] * 0.1275174307460247f) - (scores_max[1] * 0.1275174307460247f)));
    acc_s[22] = tl::fast_exp2(((acc_s[22] * 0.1275174307460247f) - (scores_max[1] * 0.1275174307460247f)));
    acc_s[23] = tl::fast_exp2(((acc_s[23] * 0.1275174307460247f) - (scores_max[1] * 0.1275174307460247f)));
    acc_s[24] = tl::fast_exp2(((acc_s[24] * 0.1275174307460247f) - (scores_max[1] * 0.1275174307460247f)));
    acc_s[25] = tl::fast_exp2(((acc_s[25] * 0.1275174307460247f) - (scores_max[1] * 0.1275174307460247f)));
    acc_s[26] = tl::fast_exp2(((acc_s[26] * 0.1275174307460247f) - (scores_max[1] * 0.1275174307460247f)));
    acc_s[27] = tl::fast_exp2(((acc_s[27] * 0.1275174307460247f) - (scores_max[1] * 0.1275174307460247f)));
    acc_s[28] = tl::fast_exp2(((acc_s[28] * 0.1275174307460247f) - (scores_max[1] * 0.1275174307460247f)));
    acc_s[29] = tl::fast_exp2(((acc_s[29] * 0.1275174307460247f) - (scores_max[1] * 0.1275174307460247f)));
    acc_s[30] = tl::fast_exp2(((acc_s[30] * 0.1275174307460247f) - (scores_max[1] * 0.1275174307460247f)));
    acc_s[31] = tl::fast_exp2(((acc_s[31] * 0.1275174307460247f) - (scores_max[1] * 0.1275174307460247f)));
    {
      const float red0_3 = ((((acc_s[0] + acc_s[1]) + (acc_s[2] + acc_s[3])) + ((acc_s[4] + acc_s[5]) + (acc_s[6] + acc_s[7]))) + (((acc_s[8] + acc_s[9]) + (acc_s[10] + acc_s[11])) + ((acc_s[12] + acc_s[13]) + (acc_s[14] + acc_s[15]))));
      const float red1_3 = ((((acc_s[16] + acc_s[17]) + (acc_s[18] + acc_s[19])) + ((acc_s[20] + acc_s[21]) + (acc_s[22] + acc_s[23]))) + (((acc_s[24] + acc_s[25]) + (acc_s[26] + acc_s[27])) + ((acc_s[28] + acc_s[29]) + (acc_s[30] + acc_s[31]))));
      const float redl0_3 = tl::lane_allreduce<tl::SumOp, 48>(red0_3);
      const float redl1_3 = tl::lane_allreduce<tl::SumOp, 48>(red1_3);
      scores_sum[0] = redl0_3;
      scores_sum[1] = redl1_3;
    }
    logsum[0] = ((logsum[0] * scores_scale[0]) + scores_sum[0]);
    logsum[1] = ((logsum[1] * scores_scale[1]) + scores_sum[1]);
    acc_s_cast[0] = ((bfloat16_t)(acc_s[0]));
    acc_s_cast[1] = ((bfloat16_t)(acc_s[1]));
    acc_s_cast[2] = ((bfloat16_t)(acc_s[2]));
    acc_s_cast[3] = ((bfloat16_t)(acc_s[3]));
    acc_s_cast[4] = ((bfloat16_t)(acc_s[4]));
    acc_s_cast[5] = ((bfloat16_t)(acc_s[5]));
    acc_s_cast[6] = ((bfloat16_t)(acc_s[6]));
    acc_s_cast[7] = ((bfloat16_t)(acc_s[7]));
    acc_s_cast[8] = ((bfloat16_t)(acc_s[8]));
    acc_s_cast[9] = ((bfloat16_t)(acc_s[9]));
    acc_s_cast[10] = ((bfloat16_t)(acc_s[10]));
    acc_s_cast[11] = ((bfloat16_t)(acc_s[11]));
    acc_s_cast[12] = ((bfloat16_t)(acc_s[12]));
    acc_s_cast[13] = ((bfloat16_t)(acc_s[13]));
    acc_s_cast[14] = ((bfloat16_t)(acc_s[14]));
    acc_s_cast[15] = ((bfloat16_t)(acc_s[15]));
    acc_s_cast[16] = ((bfloat16_t)(acc_s[16]));
    acc_s_cast[17] = ((bfloat16_t)(acc_s[17]));
    acc_s_cast[18] = ((bfloat16_t)(acc_s[18]));
    acc_s_cast[19] = ((bfloat16_t)(acc_s[19]));
    acc_s_cast[20] = ((bfloat16_t)(acc_s[20]));
    acc_s_cast[21] = ((bfloat16_t)(acc_s[21]));
    acc_s_cast[22] = ((bfloat16_t)(acc_s[22]));
    acc_s_cast[23] = ((bfloat16_t)(acc_s[23]));
    acc_s_cast[24] = ((bfloat16_t)(acc_s[24]));
    acc_s_cast[25] = ((bfloat16_t)(acc_s[25]));
    acc_s_cast[26] = ((bfloat16_t)(acc_s[26]));
    acc_s_cast[27] = ((bfloat16_t)(acc_s[27]));
    acc_s_cast[28] = ((bfloat16_t)(acc_s[28]));
    acc_s_cast[29] = ((bfloat16_t)(acc_s[29]));
    acc_s_cast[30] = ((bfloat16_t)(acc_s[30]));
    acc_s_cast[31] = ((bfloat16_t)(acc_s[31]));
  if (2 < NT) ISSUE_K(2);
  if (1 < NT) ISSUE_V(1);
  for (int t = 1; t < NT; ++t) {
    BAR();
    // matrix segment: S(t), rescale, O += P(t-1) V(t-1)
    S_GEMM(t);
    if ((rescale[0] != 0)) {
    if ((rescale[0] != 0)) {
      acc_o[0] = (acc_o[0] * scores_scale[0]);
      acc_o[1] = (acc_o[1] * scores_scale[0]);
      acc_o[2] = (acc_o[2] * scores_scale[0]);
      acc_o[3] = (acc_o[3] * scores_scale[0]);
      acc_o[4] = (acc_o[4] * scores_scale[0]);
      acc_o[5] = (acc_o[5] * scores_scale[0]);
      acc_o[6] = (acc_o[6] * scores_scale[0]);
      acc_o[7] = (acc_o[7] * scores_scale[0]);
      acc_o[8] = (acc_o[8] * scores_scale[0]);
      acc_o[9] = (acc_o[9] * scores_scale[0]);
      acc_o[10] = (acc_o[10] * scores_scale[0]);
      acc_o[11] = (acc_o[11] * scores_scale[0]);
      acc_o[12] = (acc_o[12] * scores_scale[0]);
      acc_o[13] = (acc_o[13] * scores_scale[0]);
      acc_o[14] = (acc_o[14] * scores_scale[0]);
      acc_o[15] = (acc_o[15] * scores_scale[0]);
      acc_o[16] = (acc_o[16] * scores_scale[0]);
      acc_o[17] = (acc_o[17] * scores_scale[0]);
      acc_o[18] = (acc_o[18] * scores_scale[0]);
      acc_o[19] = (acc_o[19] * scores_scale[0]);
      acc_o[20] = (acc_o[20] * scores_scale[0]);
      acc_o[21] = (acc_o[21] * scores_scale[0]);
      acc_o[22] = (acc_o[22] * scores_scale[0]);
      acc_o[23] = (acc_o[23] * scores_scale[0]);
      acc_o[24] = (acc_o[24] * scores_scale[0]);
      acc_o[25] = (acc_o[25] * scores_scale[0]);
      acc_o[26] = (acc_o[26] * scores_scale[0]);
      acc_o[27] = (acc_o[27] * scores_scale[0]);
      acc_o[28] = (acc_o[28] * scores_scale[0]);
      acc_o[29] = (acc_o[29] * scores_scale[0]);
      acc_o[30] = (acc_o[30] * scores_scale[0]);
      acc_o[31] = (acc_o[31] * scores_scale[0]);
      acc_o[32] = (acc_o[32] * scores_scale[1]);
      acc_o[33] = (acc_o[33] * scores_scale[1]);
      acc_o[34] = (acc_o[34] * scores_scale[1]);
      acc_o[35] = (acc_o[35] * scores_scale[1]);
      acc_o[36] = (acc_o[36] * scores_scale[1]);
      acc_o[37] = (acc_o[37] * scores_scale[1]);
      acc_o[38] = (acc_o[38] * scores_scale[1]);
      acc_o[39] = (acc_o[39] * scores_scale[1]);
      acc_o[40] = (acc_o[40] * scores_scale[1]);
      acc_o[41] = (acc_o[41] * scores_scale[1]);
      acc_o[42] = (acc_o[42] * scores_scale[1]);
      acc_o[43] = (acc_o[43] * scores_scale[1]);
      acc_o[44] = (acc_o[44] * scores_scale[1]);
      acc_o[45] = (acc_o[45] * scores_scale[1]);
      acc_o[46] = (acc_o[46] * scores_scale[1]);
      acc_o[47] = (acc_o[47] * scores_scale[1]);
      acc_o[48] = (acc_o[48] * scores_scale[1]);
      acc_o[49] = (acc_o[49] * scores_scale[1]);
      acc_o[50] = (acc_o[50] * scores_scale[1]);
      acc_o[51] = (acc_o[51] * scores_scale[1]);
      acc_o[52] = (acc_o[52] * scores_scale[1]);
      acc_o[53] = (acc_o[53] * scores_scale[1]);
      acc_o[54] = (acc_o[54] * scores_scale[1]);
      acc_o[55] = (acc_o[55] * scores_scale[1]);
      acc_o[56] = (acc_o[56] * scores_scale[1]);
      acc_o[57] = (acc_o[57] * scores_scale[1]);
      acc_o[58] = (acc_o[58] * scores_scale[1]);
      acc_o[59] = (acc_o[59] * scores_scale[1]);
      acc_o[60] = (acc_o[60] * scores_scale[1]);
      acc_o[61] = (acc_o[61] * scores_scale[1]);
      acc_o[62] = (acc_o[62] * scores_scale[1]);
      acc_o[63] = (acc_o[63] * scores_scale[1]);
    }
    }
    PV_GEMM(t - 1);
    tl::wait_vmcnt<0>();
    BAR();
    // vector segment: softmax(t), DMA of K(t+2) and V(t+1)
    scores_max_prev[0] = scores_max[0];
    scores_max_prev[1] = scores_max[1];
    {
      const float red0_2 = __builtin_fmaxf(__builtin_fmaxf(__builtin_fmaxf(__builtin_fmaxf(acc_s[0], acc_s[1]), __builtin_fmaxf(acc_s[2], acc_s[3])), __builtin_fmaxf(__builtin_fmaxf(acc_s[4], acc_s[5]), __builtin_fmaxf(acc_s[6], acc_s[7]))), __builtin_fmaxf(__builtin_fmaxf(__builtin_fmaxf(acc_s[8], acc_s[9]), __builtin_fmaxf(acc_s[10], acc_s[11])), __builtin_fmaxf(__builtin_fmaxf(acc_s[12], acc_s[13]), __builtin_fmaxf(acc_s[14], acc_s[15]))));
      const float red1_2 = __builtin_fmaxf(__builtin_fmaxf(__builtin_fmaxf(__builtin_fmaxf(acc_s[16], acc_s[17]), __builtin_fmaxf(acc_s[18], acc_s[19])), __builtin_fmaxf(__builtin_fmaxf(acc_s[20], acc_s[21]), __builtin_fmaxf(acc_s[22], acc_s[23]))), __builtin_fmaxf(__builtin_fmaxf(__builtin_fmaxf(acc_s[24], acc_s[25]), __builtin_fmaxf(acc_s[26], acc_s[27])), __builtin_fmaxf(__builtin_fmaxf(acc_s[28], acc_s[29]), __builtin_fmaxf(acc_s[30], acc_s[31]))));
      const float redl0_2 = tl::lane_allreduce<tl::MaxOp, 48>(red0_2);
      const float redl1_2 = tl::lane_allreduce<tl::MaxOp, 48>(red1_2);
      scores_max_prev[0] = __builtin_fmaxf(scores_max_prev[0], redl0_2);
      scores_max_prev[1] = __builtin_fmaxf(scores_max_prev[1], redl1_2);
    }
    rescale[0] = 0;
    {
      if ((((scores_max_prev[0] - scores_max[0]) * 0.1275174307460247f) > 8.0f)) {
        scores_scale[0] = tl::fast_exp2(((scores_max[0] - scores_max_prev[0]) * 0.1275174307460247f));
        scores_max[0] = scores_max_prev[0];
        rescale[0] = 1;
      } else {
        scores_scale[0] = 1.0f;
      }
    }
    {
      if ((((scores_max_prev[1] - scores_max[1]) * 0.1275174307460247f) > 8.0f)) {
        scores_scale[1] = tl::fast_exp2(((scores_max[1] - scores_max_prev[1]) * 0.1275174307460247f));
        scores_max[1] = scores_max_prev[1];
        rescale[0] = 1;
      } else {
        scores_scale[1] = 1.0f;
      }
    }
    acc_s[0] = tl::fast_exp2(((acc_s[0] * 0.1275174307460247f) - (scores_max[0] * 0.1275174307460247f)));
    acc_s[1] = tl::fast_exp2(((acc_s[1] * 0.1275174307460247f) - (scores_max[0] * 0.1275174307460247f)));
    acc_s[2] = tl::fast_exp2(((acc_s[2] * 0.1275174307460247f) - (scores_max[0] * 0.1275174307460247f)));
    acc_s[3] = tl::fast_exp2(((acc_s[3] * 0.1275174307460247f) - (scores_max[0] * 0.1275174307460247f)));
    acc_s[4] = tl::fast_exp2(((acc_s[4] * 0.1275174307460247f) - (scores_max[0] * 0.1275174307460247f)));
    acc_s[5] = tl::fast_exp2(((acc_s[5] * 0.1275174307460247f) - (scores_max[0] * 0.1275174307460247f)));
    acc_s[6] = tl::fast_exp2(((acc_s[6] * 0.1275174307460247f) - (scores_max[0] * 0.1275174307460247f)));
    acc_s[7] = tl::fast_exp2(((acc_s[7] * 0.1275174307460247f) - (scores_max[0] * 0.1275174307460247f)));
    acc_s[8] = tl::fast_exp2(((acc_s[8] * 0.1275174307460247f) - (scores_max[0] * 0.1275174307460247f)));
    acc_s[9] = tl::fast_exp2(((acc_s[9] * 0.1275174307460247f) - (scores_max[0] * 0.1275174307460247f)));
    acc_s[10] = tl::fast_exp2(((acc_s[10] * 0.1275174307460247f) - (scores_max[0] * 0.1275174307460247f)));
    acc_s[11] = tl::fast_exp2(((acc_s[11] * 0.1275174307460247f) - (scores_max[0] * 0.1275174307460247f)));
    acc_s[12] = tl::fast_exp2(((acc_s[12] * 0.1275174307460247f) - (scores_max[0] * 0.1275174307460247f)));
    acc_s[13] = tl::fast_exp2(((acc_s[13] * 0.1275174307460247f) - (scores_max[0] * 0.1275174307460247f)));
    acc_s[14] = tl::fast_exp2(((acc_s[14] * 0.1275174307460247f) - (scores_max[0] * 0.1275174307460247f)));
    acc_s[15] = tl::fast_exp2(((acc_s[15] * 0.1275174307460247f) - (scores_max[0] * 0.1275174307460247f)));
    acc_s[16] = tl::fast_exp2(((acc_s[16] * 0.1275174307460247f) - (scores_max[1] * 0.1275174307460247f)));
    acc_s[17] = tl::fast_exp2(((acc_s[17] * 0.1275174307460247f) - (scores_max[1] * 0.1275174307460247f)));
    acc_s[18] = tl::fast_exp2(((acc_s[18] * 0.1275174307460247f) - (scores_max[1] * 0.1275174307460247f)));
    acc_s[19] = tl::fast_exp2(((acc_s[19] * 0.1275174307460247f) - (scores_max[1] * 0.1275174307460247f)));
    acc_s[20] = tl::fast_exp2(((acc_s[20] * 0.1275174307460247f) - (scores_max[1] * 0.1275174307460247f)));
    acc_s[21] = tl::fast_exp2(((acc_s[21] * 0.1275174307460247f) - (scores_max[1] * 0.1275174307460247f)));
    acc_s[22] = tl::fast_exp2(((acc_s[22] * 0.1275174307460247f) - (scores_max[1] * 0.1275174307460247f)));
    acc_s[23] = tl::fast_exp2(((acc_s[23] * 0.1275174307460247f) - (scores_max[1] * 0.1275174307460247f)));
    acc_s[24] = tl::fast_exp2(((acc_s[24] * 0.1275174307460247f) - (scores_max[1] * 0.1275174307460247f)));
    acc_s[25] = tl::fast_exp2(((acc_s[25] * 0.1275174307460247f) - (scores_max[1] * 0.1275174307460247f)));
    acc_s[26] = tl::fast_exp2(((acc_s[26] * 0.1275174307460247f) - (scores_max[1] * 0.1275174307460247f)));
    acc_s[27] = tl::fast_exp2(((acc_s[27] * 0.1275174307460247f) - (scores_max[1] * 0.1275174307460247f)));
    acc_s[28] = tl::fast_exp2(((acc_s[28] * 0.1275174307460247f) - (scores_max[1] * 0.1275174307460247f)));
    acc_s[29] = tl::fast_exp2(((acc_s[29] * 0.1275174307460247f) - (scores_max[1] * 0.1275174307460247f)));
    acc_s[30] = tl::fast_exp2(((acc_s[30] * 0.1275174307460247f) - (scores_max[1] * 0.1275174307460247f)));
    acc_s[31] = tl::fast_exp2(((acc_s[31] * 0.1275174307460247f) - (scores_max[1] * 0.1275174307460247f)));
    {
      const float red0_3 = ((((acc_s[0] + acc_s[1]) + (acc_s[2] + acc_s[3])) + ((acc_s[4] + acc_s[5]) + (acc_s[6] + acc_s[7]))) + (((acc_s[8] + acc_s[9]) + (acc_s[10] + acc_s[11])) + ((acc_s[12] + acc_s[13]) + (acc_s[14] + acc_s[15]))));
      const float red1_3 = ((((acc_s[16] + acc_s[17]) + (acc_s[18] + acc_s[19])) + ((acc_s[20] + acc_s[21]) + (acc_s[22] + acc_s[23]))) + (((acc_s[24] + acc_s[25]) + (acc_s[26] + acc_s[27])) + ((acc_s[28] + acc_s[29]) + (acc_s[30] + acc_s[31]))));
      const float redl0_3 = tl::lane_allreduce<tl::SumOp, 48>(red0_3);
      const float redl1_3 = tl::lane_allreduce<tl::SumOp, 48>(red1_3);
      scores_sum[0] = redl0_3;
      scores_sum[1] = redl1_3;
    }
    logsum[0] = ((logsum[0] * scores_scale[0]) + scores_sum[0]);
    logsum[1] = ((logsum[1] * scores_scale[1]) + scores_sum[1]);
    acc_s_cast[0] = ((bfloat16_t)(acc_s[0]));
    acc_s_cast[1] = ((bfloat16_t)(acc_s[1]));
    acc_s_cast[2] = ((bfloat16_t)(acc_s[2]));
    acc_s_cast[3] = ((bfloat16_t)(acc_s[3]));
    acc_s_cast[4] = ((bfloat16_t)(acc_s[4]));
    acc_s_cast[5] = ((bfloat16_t)(acc_s[5]));
    acc_s_cast[6] = ((bfloat16_t)(acc_s[6]));
    acc_s_cast[7] = ((bfloat16_t)(acc_s[7]));
    acc_s_cast[8] = ((bfloat16_t)(acc_s[8]));
    acc_s_cast[9] = ((bfloat16_t)(acc_s[9]));
    acc_s_cast[10] = ((bfloat16_t)(acc_s[10]));
    acc_s_cast[11] = ((bfloat16_t)(acc_s[11]));
    acc_s_cast[12] = ((bfloat16_t)(acc_s[12]));
    acc_s_cast[13] = ((bfloat16_t)(acc_s[13]));
    acc_s_cast[14] = ((bfloat16_t)(acc_s[14]));
    acc_s_cast[15] = ((bfloat16_t)(acc_s[15]));
    acc_s_cast[16] = ((bfloat16_t)(acc_s[16]));
    acc_s_cast[17] = ((bfloat16_t)(acc_s[17]));
    acc_s_cast[18] = ((bfloat16_t)(acc_s[18]));
    acc_s_cast[19] = ((bfloat16_t)(acc_s[19]));
    acc_s_cast[20] = ((bfloat16_t)(acc_s[20]));
    acc_s_cast[21] = ((bfloat16_t)(acc_s[21]));
    acc_s_cast[22] = ((bfloat16_t)(acc_s[22]));
    acc_s_cast[23] = ((bfloat16_t)(acc_s[23]));
    acc_s_cast[24] = ((bfloat16_t)(acc_s[24]));
    acc_s_cast[25] = ((bfloat16_t)(acc_s[25]));
    acc_s_cast[26] = ((bfloat16_t)(acc_s[26]));
    acc_s_cast[27] = ((bfloat16_t)(acc_s[27]));
    acc_s_cast[28] = ((bfloat16_t)(acc_s[28]));
    acc_s_cast[29] = ((bfloat16_t)(acc_s[29]));
    acc_s_cast[30] = ((bfloat16_t)(acc_s[30]));
    acc_s_cast[31] = ((bfloat16_t)(acc_s[31]));
    if (t + 2 < NT) ISSUE_K(t + 2);
    if (t + 1 < NT) ISSUE_V(t + 1);
  }
#if PP
  if (wave_ < 4) BAR();
#endif
  if ((rescale[0] != 0)) {
    if ((rescale[0] != 0)) {
      acc_o[0] = (acc_o[0] * scores_scale[0]);
      acc_o[1] = (acc_o[1] * scores_scale[0]);
      acc_o[2] = (acc_o[2] * scores_scale[0]);
      acc_o[3] = (acc_o[3] * scores_scale[0]);
      acc_o[4] = (acc_o[4] * scores_scale[0]);
      acc_o[5] = (acc_o[5] * scores_scale[0]);
      acc_o[6] = (acc_o[6] * scores_scale[0]);
      acc_o[7] = (acc_o[7] * scores_scale[0]);
      acc_o[8] = (acc_o[8] * scores_scale[0]);
      acc_o[9] = (acc_o[9] * scores_scale[0]);
      acc_o[10] = (acc_o[10] * scores_scale[0]);
      acc_o[11] = (acc_o[11] * scores_scale[0]);
      acc_o[12] = (acc_o[12] * scores_scale[0]);
      acc_o[13] = (acc_o[13] * scores_scale[0]);
      acc_o[14] = (acc_o[14] * scores_scale[0]);
      acc_o[15] = (acc_o[15] * scores_scale[0]);
      acc_o[16] = (acc_o[16] * scores_scale[0]);
      acc_o[17] = (acc_o[17] * scores_scale[0]);
      acc_o[18] = (acc_o[18] * scores_scale[0]);
      acc_o[19] = (acc_o[19] * scores_scale[0]);
      acc_o[20] = (acc_o[20] * scores_scale[0]);
      acc_o[21] = (acc_o[21] * scores_scale[0]);
      acc_o[22] = (acc_o[22] * scores_scale[0]);
      acc_o[23] = (acc_o[23] * scores_scale[0]);
      acc_o[24] = (acc_o[24] * scores_scale[0]);
      acc_o[25] = (acc_o[25] * scores_scale[0]);
      acc_o[26] = (acc_o[26] * scores_scale[0]);
      acc_o[27] = (acc_o[27] * scores_scale[0]);
      acc_o[28] = (acc_o[28] * scores_scale[0]);
      acc_o[29] = (acc_o[29] * scores_scale[0]);
      acc_o[30] = (acc_o[30] * scores_scale[0]);
      acc_o[31] = (acc_o[31] * scores_scale[0]);
      acc_o[32] = (acc_o[32] * scores_scale[1]);
      acc_o[33] = (acc_o[33] * scores_scale[1]);
      acc_o[34] = (acc_o[34] * scores_scale[1]);
      acc_o[35] = (acc_o[35] * scores_scale[1]);
      acc_o[36] = (acc_o[36] * scores_scale[1]);
      acc_o[37] = (acc_o[37] * scores_scale[1]);
      acc_o[38] = (acc_o[38] * scores_scale[1]);
      acc_o[39] = (acc_o[39] * scores_scale[1]);
      acc_o[40] = (acc_o[40] * scores_scale[1]);
      acc_o[41] = (acc_o[41] * scores_scale[1]);
      acc_o[42] = (acc_o[42] * scores_scale[1]);
      acc_o[43] = (acc_o[43] * scores_scale[1]);
      acc_o[44] = (acc_o[44] * scores_scale[1]);
      acc_o[45] = (acc_o[45] * scores_scale[1]);
      acc_o[46] = (acc_o[46] * scores_scale[1]);
      acc_o[47] = (acc_o[47] * scores_scale[1]);
      acc_o[48] = (acc_o[48] * scores_scale[1]);
      acc_o[49] = (acc_o[49] * scores_scale[1]);
      acc_o[50] = (acc_o[50] * scores_scale[1]);
      acc_o[51] = (acc_o[51] * scores_scale[1]);
      acc_o[52] = (acc_o[52] * scores_scale[1]);
      acc_o[53] = (acc_o[53] * scores_scale[1]);
      acc_o[54] = (acc_o[54] * scores_scale[1]);
      acc_o[55] = (acc_o[55] * scores_scale[1]);
      acc_o[56] = (acc_o[56] * scores_scale[1]);
      acc_o[57] = (acc_o[57] * scores_scale[1]);
      acc_o[58] = (acc_o[58] * scores_scale[1]);
      acc_o[59] = (acc_o[59] * scores_scale[1]);
      acc_o[60] = (acc_o[60] * scores_scale[1]);
      acc_o[61] = (acc_o[61] * scores_scale[1]);
      acc_o[62] = (acc_o[62] * scores_scale[1]);
      acc_o[63] = (acc_o[63] * scores_scale[1]);
    }
  }
  PV_GEMM(NT - 1);
  acc_o[0] = (acc_o[0] / logsum[0]);
  acc_o[1] = (acc_o[1] / logsum[0]);
  acc_o[2] = (acc_o[2] / logsum[0]);
  acc_o[3] = (acc_o[3] / logsum[0]);
  acc_o[4] = (acc_o[4] / logsum[0]);
  acc_o[5] = (acc_o[5] / logsum[0]);
  acc_o[6] = (acc_o[6] / logsum[0]);
  acc_o[7] = (acc_o[7] / logsum[0]);
  acc_o[8] = (acc_o[8] / logsum[0]);
  acc_o[9] = (acc_o[9] / logsum[0]);
  acc_o[10] = (acc_o[10] / logsum[0]);
  acc_o[11] = (acc_o[11] / logsum[0]);
  acc_o[12] = (acc_o[12] / logsum[0]);
  acc_o[13] = (acc_o[13] / logsum[0]);
  acc_o[14] = (acc_o[14] / logsum[0]);
  acc_o[15] = (acc_o[15] / logsum[0]);
  acc_o[16] = (acc_o[16] / logsum[0]);
  acc_o[17] = (acc_o[17] / logsum[0]);
  acc_o[18] = (acc_o[18] / logsum[0]);
  acc_o[19] = (acc_o[19] / logsum[0]);
  acc_o[20] = (acc_o[20] / logsum[0]);
  acc_o[21] = (acc_o[21] / logsum[0]);
  acc_o[22] = (acc_o[22] / logsum[0]);
  acc_o[23] = (acc_o[23] / logsum[0]);
  acc_o[24] = (acc_o[24] / logsum[0]);
  acc_o[25] = (acc_o[25] / logsum[0]);
  acc_o[26] = (acc_o[26] / logsum[0]);
  acc_o[27] = (acc_o[27] / logsum[0]);
  acc_o[28] = (acc_o[28] / logsum[0]);
  acc_o[29] = (acc_o[29] / logsum[0]);
  acc_o[30] = (acc_o[30] / logsum[0]);
  acc_o[31] = (acc_o[31] / logsum[0]);
  acc_o[32] = (acc_o[32] / logsum[1]);
  acc_o[33] = (acc_o[33] / logsum[1]);
  acc_o[34] = (acc_o[34] / logsum[1]);
  acc_o[35] = (acc_o[35] / logsum[1]);
  acc_o[36] = (acc_o[36] / logsum[1]);
  acc_o[37] = (acc_o[37] / logsum[1]);
  acc_o[38] = (acc_o[38] / logsum[1]);
  acc_o[39] = (acc_o[39] / logsum[1]);
  acc_o[40] = (acc_o[40] / logsum[1]);
  acc_o[41] = (acc_o[41] / logsum[1]);
  acc_o[42] = (acc_o[42] / logsum[1]);
  acc_o[43] = (acc_o[43] / logsum[1]);
  acc_o[44] = (acc_o[44] / logsum[1]);
  acc_o[45] = (acc_o[45] / logsum[1]);
  acc_o[46] = (acc_o[46] / logsum[1]);
  acc_o[47] = (acc_o[47] / logsum[1]);
  acc_o[48] = (acc_o[48] / logsum[1]);
  acc_o[49] = (acc_o[49] / logsum[1]);
  acc_o[50] = (acc_o[50] / logsum[1]);
  acc_o[51] = (acc_o[51] / logsum[1]);
  acc_o[52] = (acc_o[52] / logsum[1]);
  acc_o[53] = (acc_o[53] / logsum[1]);
  acc_o[54] = (acc_o[54] / logsum[1]);
  acc_o[55] = (acc_o[55] / logsum[1]);
  acc_o[56] = (acc_o[56] / logsum[1]);
  acc_o[57] = (acc_o[57] / logsum[1]);
  acc_o[58] = (acc_o[58] / logsum[1]);
  acc_o[59] = (acc_o[59] / logsum[1]);
  acc_o[60] = (acc_o[60] / logsum[1]);
  acc_o[61] = (acc_o[61] / logsum[1]);
  acc_o[62] = (acc_o[62] / logsum[1]);
  acc_o[63] = (acc_o[63] / logsum[1]);
  { bfloat16_t _v[4] = {((bfloat16_t)(acc_o[0])), ((bfloat16_t)(acc_o[1])), ((bfloat16_t)(acc_o[2])), ((bfloat16_t)(acc_o[3]))}; tl::store_vec<bfloat16_t, 4>(&Output[((((bz * 33554432) + (((bx * 256) + (((((tid_ / 16) / 4) % 8) * 32) + (tid_ % 16))) * 8192)) + (by * 128)) + (((tid_ / 16) % 4) * 4))], _v); }
  { bfloat16_t _v[4] = {((bfloat16_t)(acc_o[4])), ((bfloat16_t)(acc_o[5])), ((bfloat16_t)(acc_o[6])), ((bfloat16_t)(acc_o[7]))}; tl::store_vec<bfloat16_t, 4>(&Output[((((bz * 33554432) + (((bx * 256) + (((((tid_ / 16) / 4) % 8) * 32) + (tid_ % 16))) * 8192)) + (by * 128)) + ((((tid_ / 16) % 4) * 4) + 16))], _v); }
  { bfloat16_t _v[4] = {((bfloat16_t)(acc_o[8])), ((bfloat16_t)(acc_o[9])), ((bfloat16_t)(acc_o[10])), ((bfloat16_t)(acc_o[11]))}; tl::store_vec<bfloat16_t, 4>(&Output[((((bz * 33554432) + (((bx * 256) + (((((tid_ / 16) / 4) % 8) * 32) + (tid_ % 16))) * 8192)) + (by * 128)) + ((((tid_ / 16) % 4) * 4) + 32))], _v); }
  { bfloat16_t _v[4] = {((bfloat16_t)(acc_o[12])), ((bfloat16_t)(acc_o[13])), ((bfloat16_t)(acc_o[14])), ((bfloat16_t)(acc_o[15]))}; tl::store_vec<bfloat16_t, 4>(&Output[((((bz * 33554432) + (((bx * 256) + (((((tid_ / 16) / 4) % 8) * 32) + (tid_ % 16))) * 8192)) + (by * 128)) + ((((tid_ / 16) % 4) * 4) + 48))], _v); }
  { bfloat16_t _v[4] = {((bfloat16_t)(acc_o[16])), ((bfloat16_t)(acc_o[17])), ((bfloat16_t)(acc_o[18])), ((bfloat16_t)(acc_o[19]))}; tl::store_vec<bfloat16_t, 4>(&Output[((((bz * 33554432) + (((bx * 256) + (((((tid_ / 16) / 4) % 8) * 32) + (tid_ % 16))) * 8192)) + (by * 128)) + ((((tid_ / 16) % 4) * 4) + 64))], _v); }
  { bfloat16_t _v[4] = {((bfloat16_t)(acc_o[20])), ((bfloat16_t)(acc_o[21])), ((bfloat16_t)(acc_o[22])), ((bfloat16_t)(acc_o[23]))}; tl::store_vec<bfloat16_t, 4>(&Output[((((bz * 33554432) + (((bx * 256) + (((((tid_ / 16) / 4) % 8) * 32) + (tid_ % 16))) * 8192)) + (by * 128)) + ((((tid_ / 16) % 4) * 4) + 80))], _v); }
  { bfloat16_t _v[4] = {((bfloat16_t)(acc_o[24])), ((bfloat16_t)(acc_o[25])), ((bfloat16_t)(acc_o[26])), ((bfloat16_t)(acc_o[27]))}; tl::store_vec<bfloat16_t, 4>(&Output[((((bz * 33554432) + (((bx * 256) + (((((tid_ / 16) / 4) % 8) * 32) + (tid_ % 16))) * 8192)) + (by * 128)) + ((((tid_ / 16) % 4) * 4) + 96))], _v); }
  { bfloat16_t _v[4] = {((bfloat16_t)(acc_o[28])), ((bfloat16_t)(acc_o[29])), ((bfloat16_t)(acc_o[30])), ((bfloat16_t)(acc_o[31]))}; tl::store_vec<bfloat16_t, 4>(&Output[((((bz * 33554432) + (((bx * 256) + (((((tid_ / 16) / 4) % 8) * 32) + (tid_ % 16))) * 8192)) + (by * 128)) + ((((tid_ / 16) % 4) * 4) + 112))], _v); }
  { bfloat16_t _v[4] = {((bfloat16_t)(acc_o[32])), ((bfloat16_t)(acc_o[33])), ((bfloat16_t)(acc_o[34])), ((bfloat16_t)(acc_o[35]))}; tl::store_vec<bfloat16_t, 4>(&Output[((((bz * 33554432) + (((bx * 256) + ((((((tid_ / 16) / 4) % 8) * 32) + (tid_ % 16)) + 16)) * 8192)) + (by * 128)) + (((tid_ / 16) % 4) * 4))], _v); }
  { bfloat16_t _v[4] = {((bfloat16_t)(acc_o[36])), ((bfloat16_t)(acc_o[37])), ((bfloat16_t)(acc_o[38])), ((bfloat16_t)(acc_o[39]))}; tl::store_vec<bfloat16_t, 4>(&Output[((((bz * 33554432) + (((bx * 256) + ((((((tid_ / 16) / 4) % 8) * 32) + (tid_ % 16)) + 16)) * 8192)) + (by * 128)) + ((((tid_ / 16) % 4) * 4) + 16))], _v); }
  { bfloat16_t _v[4] = {((bfloat16_t)(acc_o[40])), ((bfloat16_t)(acc_o[41])), ((bfloat16_t)(acc_o[42])), ((bfloat16_t)(acc_o[43]))}; tl::store_vec<bfloat16_t, 4>(&Output[((((bz * 33554432) + (((bx * 256) + ((((((tid_ / 16) / 4) % 8) * 32) + (tid_ % 16)) + 16)) * 8192)) + (by * 128)) + ((((tid_ / 16) % 4) * 4) + 32))], _v); }
  { bfloat16_t _v[4] = {((bfloat16_t)(acc_o[44])), ((bfloat16_t)(acc_o[45])), ((bfloat16_t)(acc_o[46])), ((bfloat16_t)(acc_o[47]))}; tl::store_vec<bfloat16_t, 4>(&Output[((((bz * 33554432) + (((bx * 256) + ((((((tid_ / 16) / 4) % 8) * 32) + (tid_ % 16)) + 16)) * 8192)) + (by * 128)) + ((((tid_ / 16) % 4) * 4) + 48))], _v); }
  { bfloat16_t _v[4] = {((bfloat16_t)(acc_o[48])), ((bfloat16_t)(acc_o[49])), ((bfloat16_t)(acc_o[50])), ((bfloat16_t)(acc_o[51]))}; tl::store_vec<bfloat16_t, 4>(&Output[((((bz * 33554432) + (((bx * 256) + ((((((tid_ / 16) / 4) % 8) * 32) + (tid_ % 16)) + 16)) * 8192)) + (by * 128)) + ((((tid_ / 16) % 4) * 4) + 64))], _v); }
  { bfloat16_t _v[4] = {((bfloat16_t)(acc_o[52])), ((bfloat16_t)(acc_o[53])), ((bfloat16_t)(acc_o[54])), ((bfloat16_t)(acc_o[55]))}; tl::store_vec<bfloat16_t, 4>(&Output[((((bz * 33554432) + (((bx * 256) + ((((((tid_ / 16) / 4) % 8) * 32) + (tid_ % 16)) + 16)) * 8192)) + (by * 128)) + ((((tid_ / 16) % 4) * 4) + 80))], _v); }
  { bfloat16_t _v[4] = {((bfloat16_t)(acc_o[56])), ((bfloat16_t)(acc_o[57])), ((bfloat16_t)(acc_o[58])), ((bfloat16_t)(acc_o[59]))}; tl::store_vec<bfloat16_t, 4>(&Output[((((bz * 33554432) + (((bx * 256) + ((((((tid_ / 16) / 4) % 8) * 32) + (tid_ % 16)) + 16)) * 8192)) + (by * 128)) + ((((tid_ / 16) % 4) * 4) + 96))], _v); }
  { bfloat16_t _v[4] = {((bfloat16_t)(acc_o[60])), ((bfloat16_t)(acc_o[61])), ((bfloat16_t)(acc_o[62])), ((bfloat16_t)(acc_o[63]))}; tl::store_vec<bfloat16_t, 4>(&Output[((((bz * 33554432) + (((bx * 256) + ((((((tid_ / 16) / 4) % 8) * 32) + (tid_ % 16)) + 16)) * 8192)) + (by * 128)) + ((((tid_ / 16) % 4) * 4) + 112))], _v); }
}
