// pbd_math.h — fp32 vector/quaternion primitives for the gfx950 kernels.
//
// Same formulas (and operand order) as the reference's `brax/math.py:25-204`
// and the jumpy helpers it uses (`brax/jumpy.py:170-192`), evaluated in fp32
// the way `jax.jit` evaluates them with x64 disabled.
#pragma once
#include <hip/hip_runtime.h>

namespace bx {

struct v3 {
  float x, y, z;
};
struct q4 {
  float w, x, y, z;
};

__device__ __forceinline__ v3 mk(float x, float y, float z) { return v3{x, y, z}; }
__device__ __forceinline__ v3 operator+(v3 a, v3 b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
__device__ __forceinline__ v3 operator-(v3 a, v3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
__device__ __forceinline__ v3 operator-(v3 a) { return {-a.x, -a.y, -a.z}; }
__device__ __forceinline__ v3 operator*(v3 a, float s) { return {a.x * s, a.y * s, a.z * s}; }
__device__ __forceinline__ v3 operator*(float s, v3 a) { return {s * a.x, s * a.y, s * a.z}; }
__device__ __forceinline__ v3 operator/(v3 a, float s) { return {a.x / s, a.y / s, a.z / s}; }
__device__ __forceinline__ v3 mul(v3 a, v3 b) { return {a.x * b.x, a.y * b.y, a.z * b.z}; }
__device__ __forceinline__ float dot(v3 a, v3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
__device__ __forceinline__ v3 cross(v3 a, v3 b) {
  return {a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x};
}
__device__ __forceinline__ float norm(v3 a) { return sqrtf(dot(a, a)); }

// jnp safe_norm: 0 when every |x_i| <= 1e-8 (allclose(x, 0), jumpy.py:183-189)
// sqrt stays correctly rounded here and in qnormalize: the bare v_sqrt_f32
// (1 ulp) turns normalised vectors' unit dot products into 1 - ulp, and
// acos near 1 magnifies that to 3.5e-4 rad (spherical joint angles at their
// reference offset, physics_legacy_test.py:494-552; measured)
// (the three |x_i| <= 1e-8 tests as one: the largest |x_i| against 1e-8, a
// v_max3_f32 with |.| modifiers and one compare instead of three compares
// and two mask ANDs)
__device__ __forceinline__ bool near_zero3(v3 a) {
  return fmaxf(fmaxf(fabsf(a.x), fabsf(a.y)), fabsf(a.z)) <= 1e-8f;
}
// 1 when any component is nonzero (a slot's contact count): the largest |x_i|
// against 0, as near_zero3
__device__ __forceinline__ float nonzero3(v3 a) {
  return fmaxf(fmaxf(fabsf(a.x), fabsf(a.y)), fabsf(a.z)) != 0.f ? 1.f : 0.f;
}
__device__ __forceinline__ float safe_norm(v3 a) {
  return near_zero3(a) ? 0.f : norm(a);
}

// safe_norm with the bare v_sqrt_f32 (<= 1 ulp) in the SINGLE-mode TU, for
// a constraint's magnitude only: c and the direction n = dx / (c + 1e-6)
// meet again in the impulse (c / w(n)) n, so the ulp cancels to first order
// and reaches the impulse through w's |n|^2 only (<= 2 ulp relative; the
// joint position and angle impulses, the contacts' friction and restitution
// impulses, whose clamps against the norm move by the same ulp)
__device__ __forceinline__ float cancel_norm(v3 a) {
#if defined(BX_TU_FAST) && !defined(BX_IEEE_CANCEL_NORM)
  return near_zero3(a) ? 0.f : __builtin_amdgcn_sqrtf(dot(a, a));
#else
  return safe_norm(a);
#endif
}

// the same bare sqrt for a direction normalised and used as a turn axis or
// lever direction, never fed to acos: its length is off by <= 1 ulp
__device__ __forceinline__ float dir_norm(v3 a) { return cancel_norm(a); }

__device__ __forceinline__ q4 operator+(q4 a, q4 b) {
  return {a.w + b.w, a.x + b.x, a.y + b.y, a.z + b.z};
}
__device__ __forceinline__ q4 operator*(q4 a, float s) { return {a.w * s, a.x * s, a.y * s, a.z * s}; }
__device__ __forceinline__ q4 operator*(float s, q4 a) { return {s * a.w, s * a.x, s * a.y, s * a.z}; }

// math.py:25-40
__device__ __forceinline__ v3 rotate(v3 v, q4 q) {
  v3 u{q.x, q.y, q.z};
  float s = q.w;
  v3 r = 2.f * (dot(u, v) * u) + (s * s - dot(u, u)) * v;
  return r + 2.f * s * cross(u, v);
}
// rotate() of several vectors by one quaternion: the same formula
// ((s^2 - |u|^2) v + 2 (u.v) u + 2 s u x v) as a matrix, built once (rows)
struct RotM {
  v3 r0, r1, r2;
};
__device__ __forceinline__ RotM rot_matrix(q4 q) {
  const float k = q.w * q.w - (q.x * q.x + q.y * q.y + q.z * q.z);
  const float tx = 2.f * q.x, ty = 2.f * q.y, tz = 2.f * q.z, ts = 2.f * q.w;
  const float xy = tx * q.y, xz = tx * q.z, yz = ty * q.z;
  const float sx = ts * q.x, sy = ts * q.y, sz = ts * q.z;
  return {{k + tx * q.x, xy - sz, xz + sy}, {xy + sz, k + ty * q.y, yz - sx},
          {xz - sy, yz + sx, k + tz * q.z}};
}
__device__ __forceinline__ v3 mrot(const RotM& m, v3 v) {
  return {dot(m.r0, v), dot(m.r1, v), dot(m.r2, v)};
}
// math.py:130-145
__device__ __forceinline__ q4 quat_mul(q4 u, q4 v) {
  return {u.w * v.w - u.x * v.x - u.y * v.y - u.z * v.z,
          u.w * v.x + u.x * v.w + u.y * v.z - u.z * v.y,
          u.w * v.y - u.x * v.z + u.y * v.w + u.z * v.x,
          u.w * v.z + u.x * v.y - u.y * v.x + u.z * v.w};
}
// math.py:148-170
__device__ __forceinline__ q4 vec_quat_mul(v3 u, q4 v) {
  return {-u.x * v.x - u.y * v.y - u.z * v.z,
          u.x * v.w + u.y * v.z - u.z * v.y,
          -u.x * v.z + u.y * v.w + u.z * v.x,
          u.x * v.y - u.y * v.x + u.z * v.w};
}
// math.py:173-187
// sin and cos of a half joint angle. Joint angles come from atan2 (clipped
// to limits), so |x| <= pi/2: Cephes' single-precision minimax polynomials
// on [-pi/4, pi/4], the upper band reflected through pi/2 - |x| (exact
// Sterbenz subtraction + 3-part Cody-Waite pi/2), <= 1.5 ulp like the
// library's; ~20 VALU instead of sincosf's 129 (its large-argument
// reduction is evaluated branch-free). Larger |x| takes the library.
__device__ __forceinline__ void sincos_half(float x, float* s, float* c) {
  const float ax = fabsf(x);
  if (ax > 1.57079637f) {
    sincosf(x, s, c);
    return;
  }
  const bool hi = ax > 0.785398163f;
  const float y = ((1.5703125f - ax) + 4.837512969970703125e-4f) + 7.54978995489188216e-8f;
  const float z = hi ? y : ax;
  const float z2 = z * z;
  const float sp =
      fmaf(fmaf(fmaf(-1.9515295891e-4f, z2, 8.3321608736e-3f), z2, -1.6666654611e-1f), z2 * z, z);
  const float cp = fmaf(
      fmaf(fmaf(fmaf(2.443315711809948e-5f, z2, -1.388731625493765e-3f), z2, 4.166664568298827e-2f),
           z2, -0.5f),
      z2, 1.f);
  *s = copysignf(hi ? cp : sp, x);
  *c = hi ? sp : cp;
}
__device__ __forceinline__ q4 quat_rot_axis(v3 axis, float angle) {
  float s, c;
  sincos_half(angle * 0.5f, &s, &c);
  return {c, axis.x * s, axis.y * s, axis.z * s};
}
__device__ __forceinline__ q4 quat_inv(q4 q) { return {q.w, -q.x, -q.y, -q.z}; }
// math.py:116-127
__device__ __forceinline__ float signed_angle(v3 axis, v3 ref_p, v3 ref_c) {
  return atan2f(dot(cross(ref_p, ref_c), axis), dot(ref_p, ref_c));
}
// a / b with the fast reciprocal's quotient corrected by one Newton step on
// the exact (fma) residual: IEEE division's correctly rounded result in all
// but rare ties, at 4 VALU instead of 2 (rcp, mul) or ~6-10 (the IEEE
// sequence); the body integration's quotients (qnormalize, vproj)
__device__ __forceinline__ float ndiv(float a, float b) {
  const float r = __builtin_amdgcn_rcpf(b);
  const float q = a * r;
  return __builtin_fmaf(__builtin_fmaf(-b, q, a), r, q);
}
__device__ __forceinline__ v3 ndiv3(v3 a, float b) {
  const float r = __builtin_amdgcn_rcpf(b);
  const v3 q = a * r;
  return mk(__builtin_fmaf(__builtin_fmaf(-b, q.x, a.x), r, q.x),
            __builtin_fmaf(__builtin_fmaf(-b, q.y, a.y), r, q.y),
            __builtin_fmaf(__builtin_fmaf(-b, q.z, a.z), r, q.z));
}
// diagnostic A/B (tools/gpu_drift_ab.sh): IEEE division inside one group of
// functions (the contacts, the body integration, the joints and actuators)
#if defined(BX_IEEE_CONTACT)
#define BX_IEEE_IN_CONTACT _Pragma("clang fp reciprocal(off)")
#else
#define BX_IEEE_IN_CONTACT
#endif
#if defined(BX_IEEE_BODY)
#define BX_IEEE_IN_BODY _Pragma("clang fp reciprocal(off)")
#else
#define BX_IEEE_IN_BODY
#endif
#if defined(BX_IEEE_JOINT)
#define BX_IEEE_IN_JOINT _Pragma("clang fp reciprocal(off)")
#else
#define BX_IEEE_IN_JOINT
#endif
// IEEE division in the legacy_spring step's impulse functions (the spring
// joints, the impulse contacts and their (1e-8 + count) reduction), always:
// with the build's fast reciprocal, legacy_spring Grasp ran 1.17x its per-env
// bound (2 x Brax's own fp32 error) and 0.6x under IEEE division; its stiff
// springs amplify the quotients' extra ulp (tests/test_gpu_parity.py)
#define BX_IEEE_IN_SPRING _Pragma("clang fp reciprocal(off)")


// A monotone stand-in for atan2(y, x) over (-pi, pi]: 1 - x / (|x| + |y|)
// for y >= 0, x / (|x| + |y|) - 1 below, (0, 0) -> 0 as atan2(0, 0). Comparing
// it with a limit's pseudo-angle decides `atan2(y, x) < limit` without the
// transcendental (the two differ only inside the rounding band of the
// boundary, where fp32 atan2 and the float64 reference differ too).
__device__ __forceinline__ float pseudo_angle(float x, float y) {
  BX_IEEE_IN_JOINT
  const float r = fabsf(x) + fabsf(y);
  const float t = r > 0.f ? x / r : 1.f;
  return y >= 0.f ? 1.f - t : t - 1.f;
}
// the Angle actuator's target act * pi / 180 (actuators.py:75-91), divided
// as jnp divides (correctly rounded), not through the build's fast
// reciprocal: the quotient is the same in every fp32 realisation of Brax (no
// state perturbation reaches it), so its extra ulp is a systematic error
// that Brax's fp32 envelope does not cover (legacy_spring Grasp ran 1.17x
// its per-env bound through its stiff Angle actuators)
__device__ __forceinline__ float deg_to_rad(float a) {
  _Pragma("clang fp reciprocal(off)")
  return a * 3.14159265358979323846f / 180.f;
}
__device__ __forceinline__ float clampf(float x, float lo, float hi) {
  return x < lo ? lo : (x > hi ? hi : x);
}

// NaN semantics under the finite-math build (`step` never
// raises, NaN / Inf propagate). The build assumes no NaN in any value it
// computed, so `x != x`, `isnan` and `x * (c ? 1 : 0)` fold to false / a
// select; the tests below see x through an empty asm (an opaque copy), so
// the compiler cannot know it is not NaN, and test its bits.
__device__ __forceinline__ bool is_nan(float x) {
  asm("" : "+v"(x));
  return (__float_as_uint(x) & 0x7fffffffu) > 0x7f800000u;
}
// 0, or a quiet NaN when x is NaN (itself opaque, so no NaN-free assumption
// removes it). The reference multiplies its contact impulses by 0 / 1 masks
// (`p = dlambda * n * coll_mask`, colliders.py:332-333; `* apply_n`,
// `* sm`): NaN * 0 is NaN, so a NaN contact's impulse is NaN where the mask
// is 0. The kernels write those masks as `c ? 1 : nan_of(pen)`.
__device__ __forceinline__ float nan_of(float x) {
  float r = is_nan(x) ? __uint_as_float(0x7fc00000u) : 0.f;
  asm("" : "+v"(r));
  return r;
}
// jnp.clip (`minimum(maximum(x, lo), hi)`): NaN for NaN (the finite-math
// clampf's min / max return the bound)
__device__ __forceinline__ float clampn(float x, float lo, float hi) {
  return is_nan(x) ? x : clampf(x, lo, hi);
}
// jp.where(x < lo, 0, 1) then jp.where(x > hi, 0, that): 1 for NaN (both
// compares false), whatever way the build rewrites the compares
__device__ __forceinline__ bool in_range_or_nan(float x, float lo, float hi) {
  return is_nan(x) || !(x < lo || x > hi);
}
__device__ __forceinline__ float signf(float x) { return (float)((x > 0.f) - (x < 0.f)); }

// q / |q| with the bare v_sqrt_f32 (the Ant env kernel's integrator only)
__device__ __forceinline__ q4 qnormalize_bare(q4 r) {
  BX_IEEE_IN_BODY
  float rn = __builtin_amdgcn_sqrtf(r.w * r.w + r.x * r.x + r.y * r.y + r.z * r.z);
  return {r.w / rn, r.x / rn, r.y / rn, r.z / rn};
}
// q / |q| (integrators.py:67, 133)
// (the quotients Newton-corrected: the fast reciprocal's extra ulp here, the
// same way at every substep, left each quaternion's norm off 1 by a bias and
// doubled Humanoid's long-horizon divergence from Brax's fp32; IEEE division
// in the body integration alone took the ratio from 2.5 to 1.0 in the A/B of
// tools/gpu_drift_ab.sh, none in the joints, contacts, pseudo-angles or
// constant quotients did)
// (every kernel but the MULTI one since round 5. `fast`: the build's fast
// quotients, the MULTI kernel's choice by measurement: on Ant Mountain its
// per-env parity ratios are the same either way (largest 0.51 fast vs 0.50
// Newton over 46 gates, tests/test_gpu_parity.py) and the Newton steps cost
// it 2 % (331 vs 325 us per 2,048-env step, tools/multi_ab.sh); the item
// loops need them: with fast quotients their per-env gate failed on legacy
// Grasp / Swimmer and the pendulums)
__device__ __forceinline__ q4 qnormalize(q4 r, bool fast = false) {
  BX_IEEE_IN_BODY
  float rn = sqrtf(r.w * r.w + r.x * r.x + r.y * r.y + r.z * r.z);
  if (fast) return {r.w / rn, r.x / rn, r.y / rn, r.z / rn};
  const float ri = __builtin_amdgcn_rcpf(rn);
  auto one = [&](float x) {
    const float q = x * ri;
    return __builtin_fmaf(__builtin_fmaf(-rn, q, x), ri, q);
  };
  return {one(r.w), one(r.x), one(r.y), one(r.z)};
}

}  // namespace bx
