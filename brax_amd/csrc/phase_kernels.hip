// phase_kernels.hip — the PBD phases as standalone HBM-streaming kernels.
//
// The fused env-step kernel keeps an env's state on chip for the whole step;
// these kernels run ONE phase over a structure-of-arrays batch instead:
//   Euler.kinetic                 integrators.py:50-68     80 B / body
//   Euler.update (acc)            integrators.py:85-93     72 B / body
//   Euler.velocity_projection     integrators.py:122-146   96 B / body
//   capsule_plane contacts        colliders.py:744-759    120 B / contact
// SoA layout: field plane k, body b, env e at base[k * plane + b * B + e]
// (env fastest), so a wavefront's 64 lanes x 4 envs read 1 KiB contiguous
// runs per field with 16-byte loads, and a contact row (fixed body a, plane
// body b) gathers its bodies' fields just as contiguously.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "pbd_launch.h"
#include "pbd_layout.h"
#include "pbd_math.h"

namespace bx {

// QP field planes in the SoA state
enum { S_POS = 0, S_ROT = 3, S_VEL = 7, S_ANG = 10, S_FIELDS = 13 };

struct f4 {
  float v[4];
};

typedef float f32x4 __attribute__((ext_vector_type(4)));

// NT = true: read-once stream (non-temporal, does not displace L2/MALL
// lines); false: lines other workgroups re-read (a contact row's bodies)
template <bool NT = true>
__device__ __forceinline__ f4 ld4v(const float* p) {
  f32x4 t;
  if (NT)
    t = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(p));
  else
    t = *reinterpret_cast<const f32x4*>(p);
  return f4{{t.x, t.y, t.z, t.w}};
}
// non-temporal streaming store (written once, not re-read by this kernel)
__device__ __forceinline__ void st4nt(float* p, const f4& a) {
  f32x4 t = {a.v[0], a.v[1], a.v[2], a.v[3]};
  __builtin_nontemporal_store(t, reinterpret_cast<f32x4*>(p));
}

// Integrator grid: x covers one body's env quads, y = body, so a body's
// constants are wave-uniform (scalar loads) and each lane owns 4 envs of it.
// One quad per lane, no grid-stride: measured faster than a capped
// grid-stride launch (A/B in DESIGN.md).
#define PHASE_LOOP_BEGIN(B)                                            \
  const int b = blockIdx.y;                                            \
  const int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;    \
  if (q < (B) / 4) {                                                   \
    const int64_t i = (int64_t)b * (B) + q * 4;

struct PhaseArgs {
  const uint32_t* blob;
  int64_t B;         // envs (multiple of 4)
  int64_t plane;     // plane stride in floats (>= N * B, multiple of 4)
  const float* in;   // state SoA (13 planes)
  float* out;        // state SoA (13 planes); may alias `in` for kinetic/update
  const float* aux;  // update: dp SoA (vel 3, ang 3 planes); vproj: prev SoA (13)
  int64_t aux_plane;
};

// Euler.kinetic: 4 envs of one body per lane
__global__ void __launch_bounds__(256) kinetic_kernel(PhaseArgs A) {
  const BlobHdr* H = reinterpret_cast<const BlobHdr*>(A.blob);
  const float h = H->h;
  PHASE_LOOP_BEGIN(A.B)
    const uint32_t* bw = A.blob + H->o_body + b * BODY_STRIDE;
    v3 pm = mk(__uint_as_float(bw[BODY_PM]), __uint_as_float(bw[BODY_PM + 1]),
               __uint_as_float(bw[BODY_PM + 2]));
    v3 rm = mk(__uint_as_float(bw[BODY_RM]), __uint_as_float(bw[BODY_RM + 1]),
               __uint_as_float(bw[BODY_RM + 2]));
    f4 s[S_FIELDS];
#pragma unroll
    for (int k = 0; k < S_FIELDS; k++) s[k] = ld4v(A.in + k * A.plane + i);
    f4 o[7];
#pragma unroll
    for (int l = 0; l < 4; l++) {
      v3 pos = mk(s[0].v[l], s[1].v[l], s[2].v[l]);
      q4 rot{s[3].v[l], s[4].v[l], s[5].v[l], s[6].v[l]};
      v3 vel = mk(s[7].v[l], s[8].v[l], s[9].v[l]);
      v3 ang = mk(s[10].v[l], s[11].v[l], s[12].v[l]);
      pos = pos + mul(vel * h, pm);
      v3 am = mul(ang, rm);
      q4 hq = (q4{0.f, am.x, am.y, am.z} * 0.5f) * h;
      q4 r = rot + quat_mul(hq, rot);
      q4 nr = qnormalize(r);
      o[0].v[l] = pos.x; o[1].v[l] = pos.y; o[2].v[l] = pos.z;
      o[3].v[l] = nr.w; o[4].v[l] = nr.x; o[5].v[l] = nr.y; o[6].v[l] = nr.z;
    }
#pragma unroll
    for (int k = 0; k < 7; k++) st4nt(A.out + k * A.plane + i, o[k]);
  }
}

// Euler.update(acc_p=dp): vel/ang planes + dp planes -> vel/ang planes
__global__ void __launch_bounds__(256) update_acc_kernel(PhaseArgs A) {
  const BlobHdr* H = reinterpret_cast<const BlobHdr*>(A.blob);
  const float h = H->h;
  const v3 g = mk(H->gx, H->gy, H->gz);
  PHASE_LOOP_BEGIN(A.B)
    const uint32_t* bw = A.blob + H->o_body + b * BODY_STRIDE;
    v3 pm = mk(__uint_as_float(bw[BODY_PM]), __uint_as_float(bw[BODY_PM + 1]),
               __uint_as_float(bw[BODY_PM + 2]));
    v3 rm = mk(__uint_as_float(bw[BODY_RM]), __uint_as_float(bw[BODY_RM + 1]),
               __uint_as_float(bw[BODY_RM + 2]));
    f4 s[6], d[6];
#pragma unroll
    for (int k = 0; k < 6; k++) {
      s[k] = ld4v(A.in + (S_VEL + k) * A.plane + i);
      d[k] = ld4v(A.aux + k * A.aux_plane + i);
    }
    f4 o[6];
#pragma unroll
    for (int l = 0; l < 4; l++) {
      v3 vel = mk(s[0].v[l], s[1].v[l], s[2].v[l]);
      v3 ang = mk(s[3].v[l], s[4].v[l], s[5].v[l]);
      v3 dv = mk(d[0].v[l], d[1].v[l], d[2].v[l]);
      v3 da = mk(d[3].v[l], d[4].v[l], d[5].v[l]);
      vel = mul(H->vexp * vel + (dv + g) * h, pm);
      ang = mul(H->aexp * ang + da * h, rm);
      o[0].v[l] = vel.x; o[1].v[l] = vel.y; o[2].v[l] = vel.z;
      o[3].v[l] = ang.x; o[4].v[l] = ang.y; o[5].v[l] = ang.z;
    }
#pragma unroll
    for (int k = 0; k < 6; k++) st4nt(A.out + (S_VEL + k) * A.plane + i, o[k]);
  }
}

// Euler.velocity_projection(qp, qp_prev): reads pos, rot and prev pos, rot;
// writes rot, vel, ang
__global__ void __launch_bounds__(256) vproj_kernel(PhaseArgs A) {
  const BlobHdr* H = reinterpret_cast<const BlobHdr*>(A.blob);
  const float h = H->h;
  PHASE_LOOP_BEGIN(A.B)
    const uint32_t* bw = A.blob + H->o_body + b * BODY_STRIDE;
    v3 pm = mk(__uint_as_float(bw[BODY_PM]), __uint_as_float(bw[BODY_PM + 1]),
               __uint_as_float(bw[BODY_PM + 2]));
    v3 rm = mk(__uint_as_float(bw[BODY_RM]), __uint_as_float(bw[BODY_RM + 1]),
               __uint_as_float(bw[BODY_RM + 2]));
    f4 s[7], p[7];
#pragma unroll
    for (int k = 0; k < 7; k++) {
      s[k] = ld4v(A.in + k * A.plane + i);
      p[k] = ld4v(A.aux + k * A.aux_plane + i);
    }
    f4 o[10];
#pragma unroll
    for (int l = 0; l < 4; l++) {
      v3 pos = mk(s[0].v[l], s[1].v[l], s[2].v[l]);
      q4 rot{s[3].v[l], s[4].v[l], s[5].v[l], s[6].v[l]};
      v3 ppos = mk(p[0].v[l], p[1].v[l], p[2].v[l]);
      q4 prot{p[3].v[l], p[4].v[l], p[5].v[l], p[6].v[l]};
      q4 nr = qnormalize(rot);
      v3 vel = mul((pos - ppos) / h, pm);
      q4 dq = quat_mul(nr, quat_inv(prot));
      v3 a = 2.f * mk(dq.x, dq.y, dq.z) / h;
      float scl = dq.w >= 0.f ? 1.f : -1.f;
      v3 ang = mul(mul(scl * rm, a), rm);
      o[0].v[l] = nr.w; o[1].v[l] = nr.x; o[2].v[l] = nr.y; o[3].v[l] = nr.z;
      o[4].v[l] = vel.x; o[5].v[l] = vel.y; o[6].v[l] = vel.z;
      o[7].v[l] = ang.x; o[8].v[l] = ang.y; o[9].v[l] = ang.z;
    }
#pragma unroll
    for (int k = 0; k < 10; k++) st4nt(A.out + (S_ROT + k) * A.plane + i, o[k]);
  }
}

// capsule_plane (colliders.py:744-759) for every capsule-plane row of the
// system: out = 10 planes of (R, B): pos 3, vel 3, normal 3, penetration
struct ContactArgs {
  const uint32_t* blob;
  int64_t B;
  int64_t plane;      // state plane stride
  const float* in;    // state SoA
  float* out;         // contact SoA
  int64_t out_plane;  // >= R * B
};

__global__ void __launch_bounds__(256) capsule_plane_kernel(ContactArgs A) {
  const BlobHdr* H = reinterpret_cast<const BlobHdr*>(A.blob);
  const int r = blockIdx.y;
  const uint32_t* rw = A.blob + H->o_row + r * ROW_STRIDE;
  if (rw[R_FN] != 0) return;  // row-uniform: capsule-capsule rows are not this kernel's
  const int a = (int)rw[R_A], pb = (int)rw[R_B];
  const v3 end = mk(__uint_as_float(rw[R_AEND]), __uint_as_float(rw[R_AEND + 1]),
                    __uint_as_float(rw[R_AEND + 2]));
  const float rad = __uint_as_float(rw[R_ARAD]);
  const int64_t quads = A.B / 4;
  for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < quads;
       q += (int64_t)gridDim.x * blockDim.x) {
    const int64_t e = q * 4;
    f4 s[S_FIELDS], t[7];
#pragma unroll
    for (int k = 0; k < S_FIELDS; k++) s[k] = ld4v<false>(A.in + k * A.plane + (int64_t)a * A.B + e);
#pragma unroll
    for (int k = 0; k < 7; k++) t[k] = ld4v<false>(A.in + k * A.plane + (int64_t)pb * A.B + e);
    f4 o[10];
#pragma unroll
    for (int l = 0; l < 4; l++) {
      v3 apos = mk(s[0].v[l], s[1].v[l], s[2].v[l]);
      q4 arot{s[3].v[l], s[4].v[l], s[5].v[l], s[6].v[l]};
      v3 avel = mk(s[7].v[l], s[8].v[l], s[9].v[l]);
      v3 aang = mk(s[10].v[l], s[11].v[l], s[12].v[l]);
      v3 bpos = mk(t[0].v[l], t[1].v[l], t[2].v[l]);
      q4 brot{t[3].v[l], t[4].v[l], t[5].v[l], t[6].v[l]};
      v3 cw = apos + rotate(end, arot);
      v3 n = rotate(mk(0.f, 0.f, 1.f), brot);
      v3 pos = cw - n * rad;
      v3 vel = avel + cross(aang, pos - apos);
      float pen = dot(bpos - pos, n);
      o[0].v[l] = pos.x; o[1].v[l] = pos.y; o[2].v[l] = pos.z;
      o[3].v[l] = vel.x; o[4].v[l] = vel.y; o[5].v[l] = vel.z;
      o[6].v[l] = n.x; o[7].v[l] = n.y; o[8].v[l] = n.z;
      o[9].v[l] = pen;
    }
#pragma unroll
    for (int k = 0; k < 10; k++) st4nt(A.out + k * A.out_plane + (int64_t)r * A.B + e, o[k]);
  }
}

hipError_t launch_phase(int which, const uint32_t* blob, int N, int64_t B, int64_t plane,
                        const float* in, float* out, const float* aux, int64_t aux_plane,
                        hipStream_t s) {
  PhaseArgs a{blob, B, plane, in, out, aux, aux_plane};
  dim3 grid((unsigned)((B / 4 + 255) / 256), (unsigned)N);
  switch (which) {
    case 0: hipLaunchKernelGGL(kinetic_kernel, grid, dim3(256), 0, s, a); break;
    case 1: hipLaunchKernelGGL(update_acc_kernel, grid, dim3(256), 0, s, a); break;
    case 2: hipLaunchKernelGGL(vproj_kernel, grid, dim3(256), 0, s, a); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

hipError_t launch_capsule_plane(const uint32_t* blob, int R, int64_t B, int64_t plane,
                                const float* in, float* out, int64_t out_plane, hipStream_t s) {
  ContactArgs a{blob, B, plane, in, out, out_plane};
  int64_t quads = B / 4;
  int64_t gx = (quads + 255) / 256;
  if (gx > 512) gx = 512;
  dim3 grid((unsigned)(gx > 0 ? gx : 1), (unsigned)R);
  hipLaunchKernelGGL(capsule_plane_kernel, grid, dim3(256), 0, s, a);
  return hipGetLastError();
}

}  // namespace bx
