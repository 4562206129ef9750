// pbd_launch.h — host-side launch entry points of pbd_kernels.hip
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/brax_amd.h"
#include "pbd_layout.h"

namespace bx {

struct StepArgs {
  const uint32_t* blob;
  int64_t n_envs;
  bx_qp qin, qout;
  const float* act;
  int64_t act_stride, act_width;
  bx_info info;
  // MULTI: the contacts of a pass's penetrating rows past MCBUF (env e's at
  // movf + e * (R - MCBUF) * MOVF_W; null when R <= MCBUF)
  float* movf;
};
struct EnvArgs {
  const uint32_t* blob;
  int64_t n_envs;
  bx_env_params P;
  bx_env_state in, out;
  const float* act;
  int64_t act_stride, act_width;
  // consecutive env steps per launch (bx_env_rollout_packed; <= 1: one step):
  // step t's action rows at act + t * act_step, its outputs at the out
  // pointers + t * out_step floats (rng + t * rng_step)
  int32_t n_steps;
  int64_t act_step, out_step, rng_step;
  // on-device action draws (bx_env_rollout_random; draw = 0: read act): step
  // t's action a of env e is uniform_at(draw_seed, draw_offset + t * draw_step
  // + e * act_width + a, draw_lo, draw_hi), the same bits as bx_uniform_slabs;
  // recorded at act_out[(t * n_envs + e) * act_width + a] when act_out is set
  int32_t draw;
  int32_t packed;  // the outputs are the packed block layout (bx_env_*_packed / rollouts)
  uint64_t draw_seed, draw_offset, draw_step;
  float draw_lo, draw_hi;
  float* act_out;
  // SINGLE mode: blob + o_lane (the lane image), so the one-step kernels
  // issue its loads before the header arrives (last: the other kernels'
  // argument offsets stay as they were)
  const uint32_t* lane_img;
  // the blob's header, for the one-step kernels: read from the arguments,
  // which the kernel holds at its start, instead of one more dependent load
  // from the blob
  BlobHdr hdr;
};
struct InfoArgs {
  const uint32_t* blob;
  int64_t n_envs;
  bx_qp q;
  bx_info info;
  int kind, obs_size, obs_flags;
  float coef[8];  // the env's bx_env_params.coef (body indices of the obs programs)
  const float* act;
  int64_t act_stride, act_width;
  float* obs;
  float* angle;  // joint angles (B, D) and velocities (B, D), or null
  float* angvel;
  // reset: env scalars written as zeros (null = skip)
  float* zero_reward;
  float* zero_done;
  float* zero_steps;
  float* zero_trunc;
  float* zero_metrics;
  int n_metrics;
};
struct ResetArgs {
  const uint32_t* blob;
  int64_t n_envs;
  const float* angle;
  const float* vel;
  bx_qp out;
  // gen = 1: angle = default_angle + U(seed, g*2D + k), vel = U(seed, g*2D + D + k)
  // with g = env_offset + e and U uniform in [-scale, scale) (angle/vel unused);
  // seeds non-null: env e uses (seeds[e], k) and (seeds[e], D + k)
  int gen;
  uint64_t seed;
  int64_t env_offset;
  const uint64_t* seeds;
  float scale;
  // gen = 1: the env kind's reset program (bx_env_reset) and its coef
  int kind;
  float coef[8];
  uint32_t* rng_out;  // UR5E / FETCH / GRASP: the per-env streams (or null)
};

// SINGLE-mode step kernels (fast-reciprocal translation unit)
hipError_t launch_system_step_single(int L, int feat, int gw, int tpb, int64_t n_envs, size_t lds,
                                     hipStream_t s, const StepArgs& a);
hipError_t launch_env_step_single(int L, int feat, int gw, int tpb, int64_t n_envs, size_t lds,
                                  hipStream_t s, const EnvArgs& a, int fold);
// MULTI-mode step kernel (large pbd scenes, L = 128 or 256 threads per env;
// jh: the joint halves)
hipError_t launch_system_step_multi(int L, int jh, int64_t n_envs, size_t lds, hipStream_t s,
                                    const StepArgs& a);
// item-loop step kernels (generic translation unit)
hipError_t launch_system_step_generic(int L, int mode, int feat, int tpb, int64_t n_envs, size_t lds,
                                      hipStream_t s, const StepArgs& a);
hipError_t launch_env_step_generic(int L, int mode, int feat, int tpb, int64_t n_envs, size_t lds,
                                   hipStream_t s, const EnvArgs& a);
hipError_t launch_info_obs(int L, int64_t n_envs, size_t lds, hipStream_t s, const InfoArgs& a);
hipError_t launch_default_qp(int64_t n_envs, size_t lds, hipStream_t s, const ResetArgs& a);
hipError_t launch_uniform(float* out, int64_t n, uint64_t seed, uint64_t offset, float lo, float hi,
                          hipStream_t s);
hipError_t launch_uniform_slabs(float* out, int64_t slab_n, int64_t n_slabs, uint64_t seed,
                                uint64_t offset, uint64_t slab_stride, const int64_t* epoch,
                                uint64_t epoch_stride, float lo, float hi, hipStream_t s);

hipError_t debug_stamps(unsigned long long* out, int reset);
hipError_t debug_partner(float* out64, int lanes, hipStream_t s);
// the feature mask F of the SINGLE-mode kernel BX_DISPATCH_SINGLE picks for
// (lanes, system features, gather width): its bit 1 (F_SPH) says whether it
// reads the LDS-staged joint limit rows
int single_kernel_feat(int L, int feat, int gw);
hipError_t debug_mstamps(unsigned long long* out, int reset);  // MULTI mode (item-loop TU)
hipError_t launch_phase(int which, const uint32_t* blob, int N, int64_t B, int64_t plane,
                        const float* in, float* out, const float* aux, int64_t aux_plane,
                        hipStream_t s);
hipError_t launch_capsule_plane(const uint32_t* blob, int R, int64_t B, int64_t plane,
                                const float* in, float* out, int64_t out_plane, hipStream_t s);

}  // namespace bx
