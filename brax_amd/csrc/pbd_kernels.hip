// pbd_kernels.hip — MI355X (gfx950) kernels of the PBD env stepper.
//
// One fused launch runs a whole `Env.step` for a batch of environments:
// `System._pbd_step` (brax/physics/system.py:254-325: actuators, joint damping,
// Euler update/kinetic, PBD joint projection, capsule contacts, velocity
// projection, contact velocity pass — `substeps` times) followed by the env
// layer (obs/reward/done/metrics, ant.py:222-282) and the Episode/AutoReset
// wrappers (wrappers.py:105-148).
//
// Work mapping: L lanes (16/32/64) of a 64-wide wavefront
// own one environment; a workgroup is one wavefront holding 64/L envs. Every
// per-item phase (bodies, joints, actuators, contact rows) spreads its items
// over the env's L lanes; the env's state lives in LDS for the whole step and
// item results are combined per body by deterministic gather lists (the
// reference's `segment_sum`s), so the only HBM traffic is the QP in/out,
// the action and the env-layer outputs.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include <type_traits>

#include "pbd_launch.h"
#include "pbd_layout.h"
#include "pbd_math.h"

// in-kernel stamps exist in the fast (SINGLE-mode) translation unit only
#if !defined(BX_TU_FAST)
#undef BX_STAMPS
#endif
// ... and the MULTI-mode ones in the item-loop translation unit only
#if !defined(BX_TU_GENERIC)
#undef BX_MSTAMPS
#endif

namespace bx {

// ---------------------------------------------------------------------------
// constant-blob accessors (the descriptor lives in HBM, read-only, L2-resident)
// ---------------------------------------------------------------------------
struct Cst {
  const uint32_t* __restrict__ w;
  __device__ __forceinline__ int i(int off) const { return (int)w[off]; }
  __device__ __forceinline__ float f(int off) const { return __uint_as_float(w[off]); }
  __device__ __forceinline__ v3 f3(int off) const { return mk(f(off), f(off + 1), f(off + 2)); }
};

struct BodyC {
  float mass;
  v3 I, pm, rm;
  q4 qm;
};
__device__ __forceinline__ BodyC load_body(const Cst& c, const BlobHdr& H, int b) {
  int o = H.o_body + b * BODY_STRIDE;
  BodyC r;
  r.mass = c.f(o + BODY_MASS);
  r.I = c.f3(o + BODY_I);
  r.pm = c.f3(o + BODY_PM);
  r.rm = c.f3(o + BODY_RM);
  r.qm = q4{c.f(o + BODY_QM), c.f(o + BODY_QM + 1), c.f(o + BODY_QM + 2), c.f(o + BODY_QM + 3)};
  return r;
}

// ---------------------------------------------------------------------------
// LDS views of one env
// ---------------------------------------------------------------------------
struct Env {
  float* qp;     // N x QP_STRIDE: pos 0..2, rot 3..6, vel 7..9, ang 10..12
  float* prev;   // N x PREV_STRIDE: pos, rot   (qprev)
  float* rb;     // N x RB_STRIDE: pos, vel, ang (qp_right_before)
  float* jslot;  // (2J + 1) x SLOT_STRIDE: parent slots, child slots, zero
  float* aslot;  // (2K + 1) x ASLOT_STRIDE
  float* rowd;   // R x ROWD_STRIDE: cpos 3, normal 3, pen, dlambda
  float* cslot;  // (2R + 1) x SLOT_STRIDE: a-side, b-side, zero
  int nJ, nK, nR;
  float* acc;    // N x 12: info contact vel 3, ang 3, info actuator ang 3, dp_a 3
  float* ang;    // 2 x D: joint angles, joint vels
  float* red;    // 64 scratch
  int* ract;     // R: NearNeighbors rank of the row this step, -1 = culled
  int* alist;    // info_rows: the step's active rows in Info order
  int sstride;   // contact slot stride: SLOT_STRIDE, or MSLOT_STRIDE in MULTI mode
  float* tslot;  // MULTI mode: (T + 1) x TSLOT_STRIDE gather-task partials, zero last
  float* nd;     // NearNeighbors candidate distances, stride nds (scratch, before the substeps)
  int nds;
  float* xact;   // the action an env program hands System.step (xact_words)
  float* arow;   // the env's action row, its first act_read words (env step)
  float* nnl;    // NearNeighbors per-wave pick lists (nnl_words)
  uint16_t* nearl;  // MULTI: the pass's near rows (in the task partials' words)
  int* nearc;       // MULTI: per-wave ballot counts (broad phase 0..15, listing 16..)
  uint32_t* bimg;   // MULTI: the rows' bounds / flags (BI_WORDS each), staged per launch
  uint16_t* sidx;   // MULTI: each row's compact contact index this pass (0xFFFF: none)
  float* cbuf;      // MULTI: the listed rows' contacts (MCBUF x MCB_W), then their rows
  uint4* cen;       // MULTI: the collidables (2 groups each)
  uint4* mat;       // MULTI: the materials (fric, elas, scale, thr)
  uint4* bod;       // MULTI: the bodies' (mass, inverse inertia), then the placed centres
  uint4* jlim;   // SINGLE spherical kernels: the lanes' limit rows, [6][L] groups
};

__device__ __forceinline__ v3 ld3(const float* p) { return mk(p[0], p[1], p[2]); }
__device__ __forceinline__ void st3(float* p, v3 v) { p[0] = v.x; p[1] = v.y; p[2] = v.z; }
__device__ __forceinline__ q4 ld4(const float* p) { return q4{p[0], p[1], p[2], p[3]}; }
__device__ __forceinline__ void st4(float* p, q4 q) { p[0] = q.w; p[1] = q.x; p[2] = q.y; p[3] = q.z; }

// 16-byte LDS accesses (ds_read_b128 / ds_write_b128) on 16-byte aligned
// records; the record strides in pbd_layout.h keep them bank-conflict-free
typedef float f32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ f32x4 ld4a(const float* p) {
  return *reinterpret_cast<const f32x4*>(__builtin_assume_aligned(p, 16));
}
__device__ __forceinline__ void st4a(float* p, f32x4 v) {
  *reinterpret_cast<f32x4*>(__builtin_assume_aligned(p, 16)) = v;
}

struct QP {
  v3 pos;
  q4 rot;
  v3 vel, ang;
};
// QP records (QP_STRIDE, 16-byte aligned): 3 x b128 + b32
__device__ __forceinline__ QP ldqp(const float* s) {
  f32x4 a = ld4a(s), b = ld4a(s + 4), c = ld4a(s + 8);
  float d = s[12];
  return QP{mk(a.x, a.y, a.z), q4{a.w, b.x, b.y, b.z}, mk(b.w, c.x, c.y), mk(c.z, c.w, d)};
}
__device__ __forceinline__ void stqp(float* s, const QP& q) {
  st4a(s, f32x4{q.pos.x, q.pos.y, q.pos.z, q.rot.w});
  st4a(s + 4, f32x4{q.rot.x, q.rot.y, q.rot.z, q.vel.x});
  st4a(s + 8, f32x4{q.vel.y, q.vel.z, q.ang.x, q.ang.y});
  s[12] = q.ang.z;
}
__device__ __forceinline__ q4 ld_rot(const float* s) {  // QP record's rot
  f32x4 a = ld4a(s), b = ld4a(s + 4);
  return q4{a.w, b.x, b.y, b.z};
}
__device__ __forceinline__ v3 ld_ang(const float* s) {  // QP record's ang
  f32x4 c = ld4a(s + 8);
  return mk(c.z, c.w, s[12]);
}
// 8-word records (slots, prev, row data): v3 at 0..2, q4 at 3..6, scalar at 7
__device__ __forceinline__ void st_slot(float* s, v3 v, q4 r, float f) {
  st4a(s, f32x4{v.x, v.y, v.z, r.w});
  st4a(s + 4, f32x4{r.x, r.y, r.z, f});
}
__device__ __forceinline__ void ld_slot(const float* s, v3& v, q4& r, float& f) {
  f32x4 a = ld4a(s), b = ld4a(s + 4);
  v = mk(a.x, a.y, a.z);
  r = q4{a.w, b.x, b.y, b.z};
  f = b.w;
}
__device__ __forceinline__ void st_v3a(float* s, v3 v) { st4a(s, f32x4{v.x, v.y, v.z, 0.f}); }
__device__ __forceinline__ v3 ld_v3a(const float* s) {
  f32x4 a = ld4a(s);
  return mk(a.x, a.y, a.z);
}
// qp_right_before records (RB_STRIDE): pos, vel, ang in 3 x b128
// a MULTI contact slot: the linear part, the angular part (3 + 3 words; slot
// k at 24 k bytes, so 8-byte accesses)
__device__ __forceinline__ void st_mslot(float* s, v3 a, v3 l) {
  float2* p = reinterpret_cast<float2*>(__builtin_assume_aligned(s, 8));
  p[0] = float2{a.x, a.y};
  p[1] = float2{a.z, l.x};
  p[2] = float2{l.y, l.z};
}
__device__ __forceinline__ void ld_mslot(const float* s, v3& a, v3& l) {
  const float2* p = reinterpret_cast<const float2*>(__builtin_assume_aligned(s, 8));
  const float2 x = p[0], y = p[1], z = p[2];
  a = mk(x.x, x.y, y.x);
  l = mk(y.y, z.x, z.y);
}

__device__ __forceinline__ void st_rb(float* s, v3 p, v3 v, v3 a) {
  st4a(s, f32x4{p.x, p.y, p.z, v.x});
  st4a(s + 4, f32x4{v.y, v.z, a.x, a.y});
  st4a(s + 8, f32x4{a.z, 0.f, 0.f, 0.f});
}
__device__ __forceinline__ void ld_rb(const float* s, v3& p, v3& v, v3& a) {
  f32x4 x = ld4a(s), y = ld4a(s + 4), z = ld4a(s + 8);
  p = mk(x.x, x.y, x.z);
  v = mk(x.w, y.x, y.y);
  a = mk(y.z, y.w, z.x);
}

// ---------------------------------------------------------------------------
// joints (brax/physics/joints.py)
// ---------------------------------------------------------------------------
struct JointC {
  int type, bp, bc, free, angle_off, n_angles, dof;
  float damping, sp, sa;
  v3 off_p, off_c;
  v3 axp[3], axc[3];
  float lim[6];
  float mp, mc;
  v3 Ip, Ic;
};
// joint halves: this lane's side of its joint (pbd_layout.h LS_*), so the
// per-substep code selects no constants by side
struct JSide {
  v3 off, ax0, ax2, I;
  float m, sg;
  int body;
};

// a revolute joint's first limit row as the hoisted kernels test it
// (pbd_layout.h LL_*): pseudo-angles and cos / sin of [lo, hi]
struct JLim {
  float plo, phi, clo, slo, chi, shi;
};

__device__ __forceinline__ JointC load_joint(const Cst& c, const BlobHdr& H, int j) {
  int o = H.o_joint + j * JOINT_STRIDE;
  JointC r;
  r.type = c.i(o + J_TYPE);
  r.bp = c.i(o + J_BP);
  r.bc = c.i(o + J_BC);
  r.free = c.i(o + J_FREE);
  r.angle_off = c.i(o + J_ANGLE_OFF);
  r.n_angles = c.i(o + J_NANGLES);
  r.dof = c.i(o + J_DOF);
  r.damping = c.f(o + J_DAMP);
  r.sp = c.f(o + J_SP);
  r.sa = c.f(o + J_SA);
  r.off_p = c.f3(o + J_OFFP);
  r.off_c = c.f3(o + J_OFFC);
  for (int k = 0; k < 3; k++) {
    r.axp[k] = c.f3(o + J_AXP + 3 * k);
    r.axc[k] = c.f3(o + J_AXC + 3 * k);
  }
  for (int k = 0; k < 6; k++) r.lim[k] = c.f(o + J_LIM + k);
  int ob = H.o_body + r.bp * BODY_STRIDE, oc = H.o_body + r.bc * BODY_STRIDE;
  r.mp = c.f(ob + BODY_MASS);
  r.mc = c.f(oc + BODY_MASS);
  r.Ip = c.f3(ob + BODY_I);
  r.Ic = c.f3(oc + BODY_I);
  return r;
}

// ---------------------------------------------------------------------------
// compile-time feature mask: kernels specialised for a system only carry the
// joint / actuator / contact kinds it uses (Ant: revolute + torque + one-way
// capsule-plane), which keeps dead paths out of the register allocation.
// ---------------------------------------------------------------------------
enum { F_SPH = 1, F_ANGLE = 2, F_CC = 4, F_TW = 8, F_FORCE = 16, F_ALL = 31 };
// F_G1 (outside F_ALL): every body's contact rows come from one collider
// group, so the per-group normalisation needs one accumulator
enum { F_G1 = 32 };
// F_X (outside F_ALL): the extended contact functions (height map, clipped
// plane, capsule-mesh, box-box SAT), item-loop kernels only. F_GEN: every
// feature, the item-loop kernels' general instantiation.
enum { F_X = 64, F_GEN = F_ALL | F_X };
// F_R2 (outside F_ALL, SINGLE mode at 16 lanes): 17-32 contact rows, lane l
// owning rows l and l + 16 (its second row's constants from the lane image's
// LI_ROW2 words)
enum { F_R2 = 256 };
// F_C16 (outside F_ALL, SINGLE mode): contact gather lists of up to 16
// entries (Pusher's wrist: 15 rows), the joint / actuator lists <= M
enum { F_C16 = 512 };
// F_R2G (with F_R2): the host put every one-way capsule-plane row in the
// lanes' first slot and every two-way capsule-capsule row in the second, so
// each slot's passes are compiled for its one contact function
enum { F_R2G = 1024 };
template <int F, int M> __device__ __forceinline__ constexpr int cl_width() {
  return (F & F_C16) ? 16 : M;
}
template <int F> __device__ __forceinline__ bool is_rev(int type) {
  if constexpr ((F & F_SPH) == 0) return true; else return type == 1;
}
template <int F> __device__ __forceinline__ bool is_torque(int type) {
  if constexpr ((F & F_ANGLE) == 0) return true; else return type == 0;
}
// F_CCO (kernel-internal): every row this code path sees is a two-way
// capsule-capsule row (F_R2G's second slot)
enum { F_CCO = 2048 };
template <int F> __device__ __forceinline__ bool is_plane(int fn) {
  if constexpr ((F & F_CCO) != 0) return false;
  else if constexpr ((F & F_CC) == 0) return true; else return fn == 0;
}
// the F_R2G kernels' two-way slot runs as contact halves (HALF: a row's a
// side on lane k, its b side on lane k + 8; the host places them so)
template <int F> __device__ __forceinline__ constexpr bool HALF() {
  return (F & F_CCO) != 0 && (F & F_R2G) != 0;
}
template <int F> __device__ __forceinline__ bool is_oneway(int ow) {
  if constexpr ((F & F_CCO) != 0) return false;
  else if constexpr ((F & F_TW) == 0) return true; else return ow != 0;
}

// Joint.apply_angle_update (joints.py:130-152): the impulse p of an angular
// correction dq; each side's rotation update is linear in it
__device__ __forceinline__ v3 angle_impulse(const JointC& J, v3 dq) {
  BX_IEEE_IN_JOINT
  float th = cancel_norm(dq);
  v3 n = dq / (th + 1e-6f);
#if defined(BX_TU_FAST)
  // w1 + w2 as one quadratic form in Ip + Ic (loop-invariant; SINGLE-mode TU)
  float dl = -th / (dot(n, mul(J.Ip + J.Ic, n)) + 1e-6f);
#else
  float w1 = dot(n, mul(J.Ip, n));
  float w2 = dot(n, mul(J.Ic, n));
  float dl = -th / (w1 + w2 + 1e-6f);
#endif
  return -dl * n;
}

// Revolute/Spherical.apply_reduced (joints.py:270-309, 332-386)
// Rodrigues' turn of v about the unit axis by the angle with (cos, sin) =
// (c, s): rotate(v, quat_rot_axis(axis, angle)) (math.py:25-40, 173-187)
__device__ __forceinline__ v3 turn(v3 v, v3 axis, float c, float s) {
  return v * c + cross(axis, v) * s + axis * (dot(axis, v) * (1.f - c));
}
// ref_p turned about the axis by the hinge angle atan2(y, x) clamped to the
// limits (math.signed_angle, joints.py:170-176): (cos, sin) is (x, y) /
// |(x, y)| inside the limits, the limit's own outside; the test on
// pseudo-angles. Neither atan2 nor the half-angle sincos is evaluated.
__device__ __forceinline__ v3 hinge_turn(v3 axis, v3 ref_p, v3 ref_c, const JLim& JL) {
  const float y = dot(cross(ref_p, ref_c), axis), x = dot(ref_p, ref_c);
  const float pa = pseudo_angle(x, y);
  const float r2 = x * x + y * y;
  // (v_rsq_f32 itself: rsqrtf's denormal-input rescaling is dead for r2 of
  // unit vectors' dot products; the same bits for every normal r2)
  const float ri = r2 > 0.f ? __builtin_amdgcn_rsqf(r2) : 0.f;
  float cph = r2 > 0.f ? x * ri : 1.f, sph = y * ri;
  cph = pa < JL.plo ? JL.clo : (pa > JL.phi ? JL.chi : cph);
  sph = pa < JL.plo ? JL.slo : (pa > JL.phi ? JL.shi : sph);
  return turn(ref_p, axis, cph, sph);
}

// A limit row (LL_*) of this lane's joint, read where it is used: the
// spherical kernels have no registers to hold three rows over the step. The
// rows are staged once per launch from the lane image (groups LI_JLIM / 4,
// + 1 and LI_JLIM12 / 4 .. + 3) into LDS as 6 slots of L lanes (stage_lim):
// li = the lane's slot-0 group, g = the row's first slot (LIM_G*). The empty
// asm keeps every use a fresh LDS read rather than a hoisted register copy.
enum { LIM_G0 = 0, LIM_G1 = 2, LIM_G2 = 4, LIM_SLOTS = 6 };
template <int L>
__device__ __forceinline__ JLim ld_lim(const uint4* li, int g) {
  asm volatile("" : "+s"(g));
  const uint4 a = li[g * L], b = li[(g + 1) * L];
  return JLim{__uint_as_float(a.x), __uint_as_float(a.y), __uint_as_float(a.z),
              __uint_as_float(a.w), __uint_as_float(b.x), __uint_as_float(b.y)};
}
// the limit cut of a torque actuator needs only the pseudo-angles
template <int L>
__device__ __forceinline__ float2 ld_lim_p(const uint4* li, int g) {
  asm volatile("" : "+s"(g));
  const uint4 a = li[g * L];
  return make_float2(__uint_as_float(a.x), __uint_as_float(a.y));
}
__device__ __forceinline__ constexpr int lim_group(int l) {
  return l == 0 ? LIM_G0 : (l == 1 ? LIM_G1 : LIM_G2);
}
// limit row `row` of a joint from its record (J_JLIM: the item-loop kernels)
__device__ __forceinline__ JLim rec_lim(const uint32_t* jrec, int row) {
  const uint32_t* r = jrec + J_JLIM + 8 * row;
  return JLim{__uint_as_float(r[LL_PLO]), __uint_as_float(r[LL_PHI]), __uint_as_float(r[LL_CLO]),
              __uint_as_float(r[LL_SLO]), __uint_as_float(r[LL_CHI]), __uint_as_float(r[LL_SHI])};
}

// JL: the hoisted kernels' limit row (pseudo-angles, cos / sin): the
// revolute hinge turn without atan2 / sincos; LI (no JL): the lane image
// whose limit rows the revolute and spherical limits read the same way;
// JREC (the item-loop kernels): the joint's record, whose J_JLIM rows they
// read the same way; none: the reference's formulas (the MULTI kernel).
// The atan2-free forms are also the more accurate: (cos, sin) of the hinge
// angle straight from (x, y) / |(x, y)|, where atan2, the half-angle sincos
// and the quaternion turn each add their ulps (the item-loop kernels' hinge
// ran 1.3-1.7x Brax's own per-env fp32 error on Acrobot / Reacher / the
// double pendulum before, tests/test_gpu_parity.py per-env gate)
template <int F, int LS = 16>
__device__ __forceinline__ void joint_apply(const JointC& J, const QP& p, const QP& c, v3& dpp, q4& dpr,
                            v3& dcp, q4& dcr, bool useJL = false, JLim JL = JLim{},
                            const uint4* LI = nullptr, const uint32_t* JREC = nullptr) {
  // each body rotates three or four of the joint's vectors: one matrix each
  BX_IEEE_IN_JOINT
  // in the SINGLE-mode TU (the item-loop / MULTI kernels keep rotate():
  // their culled Mountain scene sits closer to its gate)
#if defined(BX_TU_FAST)
  const RotM Mp = rot_matrix(p.rot), Mc = rot_matrix(c.rot);
  auto rp_ = [&](v3 v) { return mrot(Mp, v); };
  auto rc_ = [&](v3 v) { return mrot(Mc, v); };
#else
  auto rp_ = [&](v3 v) { return rotate(v, p.rot); };
  auto rc_ = [&](v3 v) { return rotate(v, c.rot); };
#endif
  // positional constraint: apply_position_update (joints.py:154-195)
  v3 pw = p.pos + rp_(J.off_p);
  v3 cw = c.pos + rc_(J.off_c);
  v3 dx = pw - cw;
  v3 rp = pw - p.pos, rc = cw - c.pos;
  float cc = cancel_norm(dx);
  v3 n = dx / (cc + 1e-6f);
  v3 cr1 = cross(rp, n), cr2 = cross(rc, n);
  float w1 = 1.f / J.mp + dot(cr1, mul(J.Ip, cr1));
  float w2 = 1.f / J.mc + dot(cr2, mul(J.Ic, cr2));
  float dl = -cc / (w1 + w2 + 1e-6f);
  v3 pv = dl * n;
  dpp = J.sp * (pv / J.mp);
  dcp = J.sp * (-pv / J.mc);
  // the angle constraints' impulses (apply_angle_update, joints.py:130-152);
  // each body's rotation update is linear in its angular impulse, so these
  // and the position constraint's add up before one quaternion product per
  // body (below)
  v3 pimp = mk(0.f, 0.f, 0.f);
  if (is_rev<F>(J.type)) {
    v3 axis = rp_(J.axp[0]);
    v3 ref_p = rp_(J.axp[2]);
    v3 ref_c = rc_(J.axc[2]);
    v3 axis_c = rc_(J.axc[0]);
    v3 dq1 = cross(axis, axis_c);
    v3 n1;
    if (useJL) {
      n1 = hinge_turn(axis, ref_p, ref_c, JL);
    } else if (LI) {
      n1 = hinge_turn(axis, ref_p, ref_c, ld_lim<LS>(LI, LIM_G0));
    } else if (JREC) {
      n1 = hinge_turn(axis, ref_p, ref_c, rec_lim(JREC, 0));
    } else {
      float psi = signed_angle(axis, ref_p, ref_c);
      float ph = clampf(psi, J.lim[0], J.lim[1]);
      q4 fix = quat_rot_axis(axis, ph);
      n1 = rotate(ref_p, fix);
    }
    v3 dq2 = cross(n1, ref_c);
    pimp = angle_impulse(J, dq1) + angle_impulse(J, dq2);
  } else {
    v3 a1p = rp_(J.axp[0]), a2p = rp_(J.axp[1]);
    v3 a1c = rc_(J.axc[0]), a2c = rc_(J.axc[1]), a3c = rc_(J.axc[2]);
    v3 lon = cross(a3c, a1p);
    lon = lon / (1e-6f + dir_norm(lon));
    v3 xz = dot(a1p, a1c) * a1c + dot(a1p, a2c) * a2c;
    xz = xz / (1e-6f + dir_norm(xz));
    v3 a2n = cross(xz, a1p);
    a2n = a2n / (1e-6f + dir_norm(a2n));
    float sg = signf(dot(a1p, a3c));
    v3 nv[3] = {a1p, -a2n * sg, a3c};
    v3 n1v[3] = {a2p, a1p, lon};
    v3 n2v[3] = {lon, xz, a2c};
    if (LI || JREC) {
      // limit_angle on pseudo-angles: inside the limits the row's impulse is
      // zero whatever the angle, outside n1 is turned by the limit's own
      // (cos, sin); neither atan2 nor sincos. The three rows' limits are
      // read first (one burst: each lane-image read is a scheduling fence,
      // ld_lim), so the three independent row chains interleave; their
      // impulses are summed in the reference's row order (Humanoid rollout
      // 32.0 -> 31.5 us per step, Env.step 42.3 -> 41.6, tools/env_ab.sh)
      JLim Lr[3];
#pragma unroll
      for (int l = 0; l < 3; l++) Lr[l] = LI ? ld_lim<LS>(LI, lim_group(l)) : rec_lim(JREC, l);
      v3 imp[3];
#pragma unroll
      for (int l = 0; l < 3; l++) {
        const JLim& L = Lr[l];
        const float y = dot(cross(n1v[l], n2v[l]), nv[l]), x = dot(n1v[l], n2v[l]);
        const float pa = pseudo_angle(x, y);
        const bool below = pa < L.plo, above = pa > L.phi;
        const v3 n1 = turn(n1v[l], nv[l], below ? L.clo : L.chi, below ? L.slo : L.shi);
        const v3 dq = cross(n1, n2v[l]) * ((below || above) ? 1.f : 0.f);
        imp[l] = angle_impulse(J, dq);
      }
      pimp = ((pimp + imp[0]) + imp[1]) + imp[2];
    }
#pragma unroll
    for (int l = 0; l < 3 && !(LI || JREC); l++) {
      // limit_angle (joints.py:343-355)
      float ph = signed_angle(nv[l], n1v[l], n2v[l]);
      float lo = J.lim[2 * l], hi = J.lim[2 * l + 1];
      float mask = ph < lo ? 1.f : 0.f;
      mask = ph > hi ? 1.f : mask;
      ph = clampf(ph, lo, hi);
      q4 fix = quat_rot_axis(nv[l], ph);
      v3 n1 = rotate(n1v[l], fix);
      v3 dq = cross(n1, n2v[l]) * mask;
      pimp = pimp + angle_impulse(J, dq);
    }
  }
  const v3 Pp = J.sp * cross(rp, pv) + J.sa * pimp;
  const v3 Pc = J.sp * cross(rc, pv) + J.sa * pimp;
  dpr = 0.5f * vec_quat_mul(mul(J.Ip, Pp), p.rot);
  dcr = -0.5f * vec_quat_mul(mul(J.Ic, Pc), c.rot);
}

// Revolute/Spherical.axis_angle (joints.py:311-319, 388-415); returns dof
template <int F>
__device__ __forceinline__ int axis_angle(const JointC& J, const QP& p, const QP& c, v3* axes, float* ang) {
  if (is_rev<F>(J.type)) {
    axes[0] = rotate(J.axp[0], p.rot);
    v3 ref_p = rotate(J.axp[2], p.rot);
    v3 ref_c = rotate(J.axc[2], c.rot);
    ang[0] = signed_angle(axes[0], ref_p, ref_c);
    return 1;
  }
  v3 a1p = rotate(J.axp[0], p.rot), a2p = rotate(J.axp[1], p.rot);
  v3 a1c = rotate(J.axc[0], c.rot), a2c = rotate(J.axc[1], c.rot), a3c = rotate(J.axc[2], c.rot);
  // (the normalisations' quotients correctly rounded, ndiv3: theta =
  // acos(cb) near cb = 1 turns the fast reciprocal's extra ulp in xz into
  // 1e-5-scale angle errors, which legacy_spring Grasp's stiff Angle
  // actuators and limit springs on its 2-dof thumb joints carried to 2.3x
  // Brax's own fp32 error, tests/test_gpu_parity.py per-env gate)
  v3 lon = cross(a3c, a1p);
  lon = ndiv3(lon, 1e-10f + safe_norm(lon));
  float psi = signed_angle(a1p, a2p, lon);
  v3 xz = dot(a1p, a1c) * a1c + dot(a1p, a2c) * a2c;
  xz = ndiv3(xz, 1e-10f + safe_norm(xz));
  float cb = dot(xz, a1p);
  float theta = acosf(clampf(cb, -1.f, 1.f)) * signf(dot(a1p, a3c)) + nan_of(cb);
  float phi = signed_angle(-a3c, a2c, lon);
  axes[0] = a1p; axes[1] = a2c; axes[2] = a3c;
  ang[0] = psi; ang[1] = theta; ang[2] = phi;
  // spring Universal.axis_angle (spring_joints.py:188-216): (psi, theta)
  return J.type == BX_JOINT_UNIVERSAL ? 2 : 3;
}

// ---------------------------------------------------------------------------
// legacy_spring joints (brax/physics/spring_joints.py)
// ---------------------------------------------------------------------------
struct SpringC {
  float stiff, sdamp, lstr;
};
__device__ __forceinline__ SpringC load_spring(const Cst& c, const BlobHdr& H, int j) {
  int o = H.o_joint + j * JOINT_STRIDE;
  return SpringC{c.f(o + J_STIFF), c.f(o + J_SDAMP), c.f(o + J_LSTR)};
}

// Revolute/Universal/Spherical.apply_reduced (spring_joints.py:122-155,
// 170-204, 262-287): the offset spring-damper impulse through Body.impulse
// (bodies.py:46-59), then the alignment / limit torques and the joint's
// angular damping. Outputs dP of parent and child (vel, ang).
__device__ __forceinline__ void spring_joint_apply(const JointC& J, const SpringC& S, const QP& p,
                                                   const QP& c, v3& dvp, v3& dap, v3& dvc,
                                                   v3& dac) {
  BX_IEEE_IN_SPRING
  // QP.to_world (base.py:110-124)
  v3 op = rotate(J.off_p, p.rot), oc = rotate(J.off_c, c.rot);
  v3 pos_p = p.pos + op, vel_p = p.vel + cross(p.ang, op);
  v3 pos_c = c.pos + oc, vel_c = c.vel + cross(c.ang, oc);
  v3 imp = (pos_p - pos_c) * S.stiff + S.sdamp * (vel_p - vel_c);
  v3 nimp = -imp;
  dvp = nimp / J.mp;
  dap = mul(J.Ip, cross(pos_p - p.pos, nimp));
  dvc = imp / J.mc;
  dac = mul(J.Ic, cross(pos_c - c.pos, imp));
  v3 axes[3];
  float ang[3];
  const int dof = axis_angle<F_ALL>(J, p, c, axes, ang);
  float dang[3];
#pragma unroll
  for (int l = 0; l < 3; l++) {
    const float lo = J.lim[2 * l], hi = J.lim[2 * l + 1];
    float d = ang[l] < lo ? lo - ang[l] : 0.f;
    dang[l] = ang[l] > hi ? hi - ang[l] : d;
  }
  v3 tq;
  if (J.type == BX_JOINT_REVOLUTE) {
    v3 axis_c = rotate(J.axc[0], c.rot);
    tq = S.stiff * cross(axes[0], axis_c);
    tq = tq - (S.lstr * axes[0]) * dang[0];
  } else if (dof == 2) {
    v3 proj = axes[1] - dot(axes[1], axes[0]) * axes[0];
    proj = proj / safe_norm(proj);
    tq = (S.lstr / 5.f) * cross(proj, axes[1]);
    tq = tq - S.lstr * (axes[0] * dang[0] + axes[1] * dang[1]);
  } else {
    tq = -S.lstr * ((axes[0] * dang[0] + axes[1] * dang[1]) + axes[2] * dang[2]);
  }
  tq = tq - J.damping * (p.ang - c.ang);
  dap = dap + mul(J.Ip, tq);
  dac = dac + mul(-J.Ic, tq);
}

// ---------------------------------------------------------------------------
// actuators (brax/physics/actuators.py:52-112)
// ---------------------------------------------------------------------------
struct ActC {
  int type, joint;
  int idx[3];
  float strength;
};
__device__ __forceinline__ ActC load_act(const Cst& c, const BlobHdr& H, int a) {
  int o = H.o_act + a * ACT_STRIDE;
  ActC r;
  r.type = c.i(o + A_TYPE);
  r.joint = c.i(o + A_JOINT);
  for (int k = 0; k < 3; k++) r.idx[k] = c.i(o + A_IDX + k);
  r.strength = c.f(o + A_STR);
  return r;
}

// ---------------------------------------------------------------------------
// contacts (brax/physics/colliders.py)
// ---------------------------------------------------------------------------
// jp.take(act, index) with mode='clip' (jumpy.py:146-151): -1 -> 0, >= width -> last
__device__ __forceinline__ int take_idx(int i, int w) { return i < 0 ? 0 : (i >= w ? w - 1 : i); }

// dp_f of body b (forces.py:41-107), constant over a step: Thruster
// dvel = a * strength / mass, Twister dang = a * strength / mass (the body's
// MASS, forces.py:85), each segment-summed over the body in application order
__device__ __forceinline__ void body_forces(const Cst& c, const BlobHdr& H, int b, const float* act,
                                            int aw, bool valid, v3& fv, v3& fa) {
  fv = mk(0.f, 0.f, 0.f);
  fa = mk(0.f, 0.f, 0.f);
  for (int f = 0; f < H.NF; f++) {
    const int o = H.o_force + f * FORCE_STRIDE;
    if (c.i(o + F_BODY) != b) continue;
    const float st = c.f(o + F_STR), m = c.f(o + F_MASS);
    v3 a = mk(0.f, 0.f, 0.f);
    if (valid)
      a = mk(act[take_idx(c.i(o + F_IDX), aw)], act[take_idx(c.i(o + F_IDX + 1), aw)],
             act[take_idx(c.i(o + F_IDX + 2), aw)]);
    v3 d = mk(a.x * st / m, a.y * st / m, a.z * st / m);
    if (c.i(o + F_TYPE) == BX_FORCE_THRUSTER) fv = fv + d;
    else fa = fa + d;
  }
}

struct RowC {
  int group, a, b, fn, oneway;
  v3 a_pos, a_end, b_pos, b_end;
  float a_rad, b_rad, fric, elas, scale, thr;
  // erp (the legacy_spring impulse model) or, in the MULTI kernel (pbd only:
  // no erp), the b side's contact slot from its row image: one register
  // either way (a separate field took the MULTI kernel past 128 VGPRs, and
  // its 256-thread workgroups from three per CU to one: tools/multi_occ.py)
  union {
    float erp;
    int bslot;
  };
  float ma, mb;
  v3 Ia, Ib;
};
__device__ __forceinline__ RowC load_row(const Cst& c, const BlobHdr& H, int r) {
  int o = H.o_row + r * ROW_STRIDE;
  RowC x;
  x.group = c.i(o + R_GROUP);
  x.a = c.i(o + R_A);
  x.b = c.i(o + R_B);
  x.fn = c.i(o + R_FN);
  x.oneway = c.i(o + R_ONEWAY);
  x.a_pos = c.f3(o + R_APOS);
  x.a_end = c.f3(o + R_AEND);
  x.a_rad = c.f(o + R_ARAD);
  x.b_pos = c.f3(o + R_BPOS);
  x.b_end = c.f3(o + R_BEND);
  x.b_rad = c.f(o + R_BRAD);
  x.fric = c.f(o + R_FRIC);
  x.elas = c.f(o + R_ELAS);
  x.scale = c.f(o + R_SCALE);
  x.thr = c.f(o + R_THR);
  x.erp = c.f(o + R_ERP);
  int oa = H.o_body + x.a * BODY_STRIDE, ob = H.o_body + x.b * BODY_STRIDE;
  x.ma = c.f(oa + BODY_MASS);
  x.mb = c.f(ob + BODY_MASS);
  x.Ia = c.f3(oa + BODY_I);
  x.Ib = c.f3(ob + BODY_I);
  return x;
}

// closest_segment_point_and_dist (geometry.py:360-374): returns dist^2
__device__ __forceinline__ float seg_point(v3 a, v3 b, v3 pt, v3& out) {
  v3 ab = b - a;
  float t = clampf(dot(pt - a, ab) / (dot(ab, ab) + 1e-6f), 0.f, 1.f);
  out = a + t * ab;
  v3 v = pt - out;
  return dot(v, v);
}

// _closest_segment_to_segment_points (geometry.py:394-451)
__device__ __forceinline__ void seg_seg(v3 a0, v3 a1, v3 b0, v3 b1, v3& ba, v3& bb) {
  v3 da = a1 - a0;
  float la = safe_norm(da);
  la += 1e-6f * (float)(la == 0.f);
  da = da / la;
  float hla = la * 0.5f;
  v3 db = b1 - b0;
  float lb = safe_norm(db);
  lb += 1e-6f * (float)(lb == 0.f);
  db = db / lb;
  float hlb = lb * 0.5f;
  v3 am = a0 + da * hla, bm = b0 + db * hlb;
  v3 tr = am - bm;
  float dadb = dot(da, db), datr = dot(da, tr), dbtr = dot(db, tr);
  float den = 1.f - dadb * dadb;
  float ota = (-datr + dadb * dbtr) / (den + 1e-6f);
  float otb = dbtr + ota * dadb;
  float ta = clampf(ota, -hla, hla), tb = clampf(otb, -hlb, hlb);
  ba = am + da * ta;
  bb = bm + db * tb;
  v3 na, nb;
  float d1 = seg_point(a0, a1, bb, na);
  float d2 = seg_point(b0, b1, ba, nb);
  if (d1 < d2) ba = na; else bb = nb;
}

// capsule_plane (colliders.py:744-759) / capsule_capsule (:805-819)
template <int F>
__device__ __forceinline__ void contact_gen(const RowC& R, const QP& a, const QP& b, v3& pos, v3& vel, v3& n,
                            float& pen) {
  if (is_plane<F>(R.fn)) {
  BX_IEEE_IN_CONTACT
    v3 e = a.pos + rotate(R.a_end, a.rot);
    n = rotate(mk(0.f, 0.f, 1.f), b.rot);
    pos = e - n * R.a_rad;
    vel = a.vel + cross(a.ang, pos - a.pos);
    pen = dot(b.pos - pos, n);
    return;
  }
  v3 pa = a.pos + rotate(R.a_pos, a.rot), ea = rotate(R.a_end, a.rot);
  v3 pb = b.pos + rotate(R.b_pos, b.rot), eb = rotate(R.b_end, b.rot);
  v3 a0 = pa + ea, a1 = pa - ea, b0 = pb + eb, b1 = pb - eb;
  v3 ba, bb;
  seg_seg(a0, a1, b0, b1, ba, bb);
  v3 pv = ba - bb;
  float dist = safe_norm(pv);
  n = pv / (1e-6f + dist);
  // (+ NaN for NaN segments: jnp's safe_norm is NaN there, allclose(NaN, 0)
  // being False; the finite-math near-zero test would return 0)
  pen = R.a_rad + R.b_rad - dist + nan_of(dot(pv, pv));
  pos = (ba + bb) / 2.f;
  vel = (a.vel + cross(a.ang, pos - a.pos)) - (b.vel + cross(b.ang, pos - b.pos));
}

// ---- extended contact functions (item-loop kernels only) -----------------

__device__ __forceinline__ float pdiv(float a, float b) { return (float)((double)a / (double)b); }

// box_heightmap, one box corner (colliders.py:699-739); height indices as
// under jit: a negative index wraps once, then the gather clamps
__device__ __noinline__ void heightmap_contact(const Cst& c, const BlobHdr& H, int o, const RowC& R,
                                               const QP& a, const QP& b, v3& pos, v3& vel, v3& n,
                                               float& pen) {
  const float cell = c.f(o + R_X);
  const int off = H.o_hm + c.i(o + R_HM_OFF), M = c.i(o + R_HM_M);
  v3 r = rotate(R.a_end, a.rot);
  pos = a.pos + r;
  vel = a.vel + cross(a.ang, r);
  v3 p = rotate(pos - b.pos, quat_inv(b.rot));
  // the grid position and the tilted-triangle normal carry no later
  // correction: divide correctly rounded here (the build's a * rcp(b) is ~1.5
  // ulp; the double quotient rounds to the fp32 IEEE one)
  float u = pdiv(p.x, cell), v = pdiv(p.y, cell);
  float fu = floorf(u), fv = floorf(v);
  int iu = (int)fu, iv = (int)fv;
  bool lower = ((u - fu) + (v - fv)) < 1.f;
  float mu = lower ? -1.f : 1.f;
  int tu[3] = {iu + (lower ? 0 : 1), iu + (lower ? 1 : 0), iu + (lower ? 0 : 1)};
  int tv[3] = {iv + (lower ? 0 : 1), iv + (lower ? 0 : 1), iv + (lower ? 1 : 0)};
  float hh[3];
#pragma unroll
  for (int k = 0; k < 3; k++) {
    int i = tu[k], j = -tv[k];
    i += i < 0 ? M : 0;
    j += j < 0 ? M : 0;
    i = i < 0 ? 0 : (i >= M ? M - 1 : i);
    j = j < 0 ? 0 : (j >= M ? M - 1 : j);
    hh[k] = c.f(off + i * M + j);
  }
  v3 raw = mk(mu * (hh[1] - hh[0]), mu * (hh[2] - hh[0]), cell);
  const float rn = safe_norm(raw);
  v3 n0 = mk(pdiv(raw.x, rn), pdiv(raw.y, rn), pdiv(raw.z, rn));
  v3 p0 = mk((float)tu[0] * cell, (float)tv[0] * cell, hh[0]);
  pen = dot(p0 - p, n0);
  n = rotate(n0, b.rot);
}

// capsule_clippedplane, one capsule end (colliders.py:762-802)
__device__ __noinline__ void clipped_contact(const Cst& c, int o, const RowC& R, const QP& a,
                                             const QP& b, v3& pos, v3& vel, v3& n, float& pen) {
  v3 e = a.pos + rotate(R.a_end, a.rot);
  v3 nb = rotate(c.f3(o + R_X), b.rot);
  float ndir = dot(a.pos, nb) > 0.f ? 1.f : -1.f;
  n = nb * ndir;
  pos = e - n * R.a_rad;
  vel = a.vel + cross(a.ang, pos - a.pos);
  v3 pt = rotate(c.f3(o + R_X + 9), b.rot) + b.pos;
  pen = dot(pt - pos, n);
  v3 nx = rotate(c.f3(o + R_X + 3), b.rot), ny = rotate(c.f3(o + R_X + 6), b.rot);
  const float hx = c.f(o + R_X + 12), hy = c.f(o + R_X + 13);
  v3 nn = n * ndir;
  v3 yn = cross(nn, nx), xn = -cross(nn, ny);
  bool front = dot(pos - (pt + nx * hx), xn) > 1e-6f;
  front |= dot(pos - (pt - nx * hx), -xn) > 1e-6f;
  front |= dot(pos - (pt + ny * hy), yn) > 1e-6f;
  front |= dot(pos - (pt - ny * hy), -yn) > 1e-6f;
  if (front) pen = -1.f;
}

// closest_triangle_point (geometry.py:462-498)
__device__ __forceinline__ v3 tri_point(v3 p0, v3 p1, v3 p2, v3 pt) {
  v3 e0 = p1 - p0, e1 = p2 - p0, d = pt - p0;
  float a = dot(e0, e0), bb = dot(e0, e1), cc = dot(e1, e1);
  float det = a * cc - bb * bb;
  float u = (cc * dot(e0, d) - bb * dot(e1, d)) / det;
  float v = (-bb * dot(e0, d) + a * dot(e1, d)) / det;
  bool inside = (0.f <= u) & (u <= 1.f) & (0.f <= v) & (v <= 1.f) & (u + v <= 1.f);
  v3 cp = p0 + u * e0 + v * e1;
  v3 w = cp - pt;
  float d0 = dot(w, w);
  v3 c1, c2, c3;
  float d1 = seg_point(p0, p1, pt, c1);
  bool use0 = (d0 < d1) & inside;
  v3 best = use0 ? cp : c1;
  float md = use0 ? d0 : d1;
  float d2 = seg_point(p1, p2, pt, c2);
  if (d2 < md) best = c2;
  md = fminf(md, d2);
  float d3 = seg_point(p2, p0, pt, c3);
  if (d3 < md) best = c3;
  return best;
}

// capsule_mesh, one triangle of a box / mesh (colliders.py:822-848) with
// closest_segment_triangle_points (geometry.py:501-541)
__device__ __noinline__ void capsule_mesh_contact(const Cst& c, int o, const RowC& R, const QP& a,
                                                  const QP& b, v3& pos, v3& vel, v3& n,
                                                  float& pen) {
  v3 pa = a.pos + rotate(R.a_pos, a.rot), ea = rotate(R.a_end, a.rot);
  v3 s0 = pa + ea, s1 = pa - ea;
  v3 tn = rotate(c.f3(o + R_X + 9), b.rot);
  v3 p0 = b.pos + rotate(c.f3(o + R_X), b.rot);
  v3 p1 = b.pos + rotate(c.f3(o + R_X + 3), b.rot);
  v3 p2 = b.pos + rotate(c.f3(o + R_X + 6), b.rot);
  v3 sp[4], tp[4];
  seg_seg(s0, s1, p0, p1, sp[0], tp[0]);
  seg_seg(s0, s1, p1, p2, sp[1], tp[1]);
  seg_seg(s0, s1, p0, p2, sp[2], tp[2]);
  {  // closest_segment_point_plane (geometry.py:377-391)
    v3 ab = s1 - s0;
    float t = (dot(p0, tn) - dot(tn, s0)) / (dot(tn, ab) + 1e-6f);
    sp[3] = s0 + clampf(t, 0.f, 1.f) * ab;
  }
  tp[3] = tri_point(p0, p1, p2, sp[3]);
  float dd[4];
#pragma unroll
  for (int i = 0; i < 4; i++) {
    v3 w = sp[i] - tp[i];
    dd[i] = dot(w, w);
  }
  float md = fminf(fminf(dd[0], dd[1]), fminf(dd[2], dd[3]));
  v3 ss = mk(0.f, 0.f, 0.f), ts = mk(0.f, 0.f, 0.f);
  float cnt = 0.f;
#pragma unroll
  for (int i = 0; i < 4; i++) {
    float m = dd[i] == md ? 1.f : 0.f;
    ss = ss + sp[i] * m;
    ts = ts + tp[i] * m;
    cnt += m;
  }
  ss = ss / cnt;
  ts = ts / cnt;
  v3 pv = ss - ts;
  float dist = safe_norm(pv);
  n = pv / (1e-6f + dist);
  pen = R.a_rad - dist;
  pos = ts;
  vel = (a.vel + cross(a.ang, pos - a.pos)) - (b.vel + cross(b.ang, pos - b.pos));
}

// ---- hull_hull: separating axis test between two boxes ---------------------
// (colliders.py:851-888; geometry.py:580-914). Every row of a pair computes
// the whole test and keeps its own contact e (4 rows a pair).
// Divisions here are correctly rounded (pdiv), whatever the TU's flags, as
// a guard: the edge contact is valid only for barycentric t in [0, 1], and
// t = (ota + la/2) / la is exactly 1 for a closest point at an edge end,
// where v_rcp_f32 + multiply could overshoot to 1 + ulp. (The BoxBoxTest
// step-8 mismatch measured on the MI355X was the exact-equality test of the
// support vertex against face-edge endpoints; hull_world fixes that below.)
__device__ __forceinline__ v3 pdiv3(v3 a, float b) { return mk(pdiv(a.x, b), pdiv(a.y, b), pdiv(a.z, b)); }
struct HullW {
  v3 v[8];
  v3 f[6][4];
  v3 n[6];
};

__device__ void hull_world(const Cst& c, const BlobHdr& H, int h, const QP& q, HullW& w) {
  const int o = H.o_hull + h * HULL_STRIDE;
  for (int i = 0; i < 8; i++) w.v[i] = q.pos + rotate(c.f3(o + HULL_V + 3 * i), q.rot);
  // a face corner that is a hull vertex takes that vertex's world point bit
  // for bit: the edge support test compares face-edge endpoints with the
  // support vertex for exact equality (geometry.py:812-814), which holds in
  // the reference because both come out of the same rotate; two separately
  // scheduled (FMA-contracted) rotates here may differ in the last ulp
  for (int f = 0; f < 6; f++) {
    w.n[f] = rotate(c.f3(o + HULL_N + 3 * f), q.rot);
    for (int i = 0; i < 4; i++) {
      const v3 fc = c.f3(o + HULL_F + 12 * f + 3 * i);
      int m = -1;
      for (int v = 0; v < 8; v++) {
        const v3 bv = c.f3(o + HULL_V + 3 * v);
        if (bv.x == fc.x && bv.y == fc.y && bv.z == fc.z) m = v;
      }
      w.f[f][i] = m >= 0 ? w.v[m] : q.pos + rotate(fc, q.rot);
    }
  }
}

// get_face_support (geometry.py:794-801)
__device__ float hull_face_support(const v3* verts, const v3* normals, const v3 (*faces)[4], int& idx) {
  float best = 0.f;
  for (int f = 0; f < 6; f++) {
    float mn = 0.f;
    for (int v = 0; v < 8; v++) {
      float x = dot(normals[f], verts[v] - faces[f][0]);
      mn = (v == 0 || x < mn) ? x : mn;
    }
    if (f == 0 || mn > best) { best = mn; idx = f; }
  }
  return best;
}

// _clip_edge_to_planes (geometry.py:580-624) against 4 planes; returns the mask
__device__ bool hull_clip_edge(v3 p0, v3 p1, const v3* pp, const v3* pn, v3& o0, v3& o1) {
  bool f0[4], f1[4];
  v3 cand[4];
  for (int j = 0; j < 4; j++) {
    f0[j] = dot(p0 - pp[j], pn[j]) > 1e-6f;
    f1[j] = dot(p1 - pp[j], pn[j]) > 1e-6f;
    v3 ab = p1 - p0;
    float t = pdiv(dot(pp[j], pn[j]) - dot(pn[j], p0), dot(pn[j], ab) + 1e-6f);
    cand[j] = p0 + clampf(t, 0.f, 1.f) * ab;
  }
  for (int side = 0; side < 2; side++) {
    const v3 a = side == 0 ? p0 : p1, b = side == 0 ? p1 : p0;
    const bool* fr = side == 0 ? f0 : f1;
    int best = 0;
    float bd = 0.f;
    for (int j = 0; j < 4; j++) {
      float d = dot((fr[j] ? cand[j] : a) - a, b - a);
      if (j == 0 || d > bd) { bd = d; best = j; }
    }
    v3 r = fr[best] ? cand[best] : a;
    if (side == 0) o0 = r; else o1 = r;
  }
  bool both = false;
  for (int j = 0; j < 4; j++) both |= f0[j] && f1[j];
  bool mask = !both;
  if (!mask) { o0 = p0; o1 = p1; }
  if (dot(p0 - p1, o0 - o1) < 0.f) mask = false;
  return mask;
}

// _create_sat_contact_manifold + clip (geometry.py:627-747): contact e
__device__ void hull_manifold(const v3* cp, const v3* sp, v3 cn, v3 sn, float sign, int e, v3& pos,
                              v3& nrm, float& pen) {
  v3 c0[4], cpn[4], s0[4], spn[4];
  for (int i = 0; i < 4; i++) {
    const int im = (i + 3) & 3;  // jp.roll(poly, 1)
    c0[i] = cp[im];
    cpn[i] = cross(cn, cp[i] - c0[i]);
    s0[i] = sp[im];
    spn[i] = cross(sn, sp[i] - s0[i]);
  }
  v3 pts[16];
  bool msk[16];
  for (int i = 0; i < 4; i++) {
    bool m = hull_clip_edge(s0[i], sp[i], c0, cpn, pts[2 * i], pts[2 * i + 1]);
    msk[2 * i] = msk[2 * i + 1] = m;
  }
  const float dd = dot(sp[0], sn), den = dot(cn, sn);
  const float dn = den + 1e-6f * (float)(den == 0.f);
  for (int i = 0; i < 4; i++) {
    v3 a = c0[i] + pdiv(dd - dot(c0[i], sn), dn) * cn;
    v3 b = cp[i] + pdiv(dd - dot(cp[i], sn), dn) * cn;
    bool m = hull_clip_edge(a, b, s0, spn, pts[8 + 2 * i], pts[8 + 2 * i + 1]);
    msk[8 + 2 * i] = msk[8 + 2 * i + 1] = m;
  }
  const v3 nh = pdiv3(cn, 1e-6f + safe_norm(cn));
  v3 ref[16];
  for (int i = 0; i < 16; i++) {
    v3 d = pts[i] - cp[0];
    ref[i] = pts[i] - dot(d, nh) * nh;
    msk[i] = msk[i] && (dot(d, -cn) > 1e-6f);
  }
  // get_orthogonals (geometry.py:568-577)
  float ca[3] = {fabsf(cn.x), fabsf(cn.y), fabsf(cn.z)};
  int ix = 0;
  for (int k = 1; k < 3; k++) if (ca[k] > ca[ix]) ix = k;
  const float cix = ix == 0 ? cn.x : (ix == 1 ? cn.y : cn.z);
  const float denom = cix + 1e-6f * (float)(cix == 0.f);
  const float bv = pdiv(-(((cn.x + cn.y) + cn.z) - cix), denom);
  v3 o1 = mk(ix == 0 ? bv : 1.f, ix == 1 ? bv : 1.f, ix == 2 ? bv : 1.f);
  v3 o2 = cross(cn, o1);
  v3 dir = e == 0 ? o1 : (e == 1 ? -o1 : (e == 2 ? o2 : -o2));
  int best = 0;
  float bvv = 0.f;
  for (int i = 0; i < 16; i++) {
    float v = dot(ref[i], dir) + (msk[i] ? 0.f : -1e6f);
    if (i == 0 || v > bvv) { bvv = v; best = i; }
  }
  pos = ref[best];
  nrm = sign * cn;
  pen = msk[best] ? dot(pts[best] - ref[best], -cn) : -1.f;
}

__device__ __noinline__ void hull_contact(const Cst& c, const BlobHdr& H, int o, const QP& a,
                                          const QP& b, v3& pos, v3& vel, v3& n, float& pen) {
  const int ha = (int)c.f(o + R_X), hb = (int)c.f(o + R_X + 1), e = (int)c.f(o + R_X + 2);
  HullW A, B;
  hull_world(c, H, ha, a, A);
  hull_world(c, H, hb, b, B);
  v3 origin = mk(0.f, 0.f, 0.f);
  for (int v = 0; v < 8; v++) origin = origin + A.v[v];
  origin = origin / 8.f;
  int i1 = 0, i2 = 0;
  const float d1 = hull_face_support(A.v, B.n, B.f, i1);
  const float d2 = hull_face_support(B.v, A.n, A.f, i2);
  const bool use_b = d1 > d2;
  const float face_dist = use_b ? d1 : d2;
  const int fi = use_b ? i1 : i2;
  const v3* ref_face = use_b ? B.f[fi] : A.f[fi];
  const v3 ref_n = use_b ? B.n[fi] : A.n[fi];
  const v3 (*inc_faces)[4] = use_b ? A.f : B.f;
  const v3* inc_ns = use_b ? A.n : B.n;
  int ii = 0;
  float bd = 0.f;
  for (int f = 0; f < 6; f++) {
    float d = dot(inc_ns[f], ref_n);
    if (f == 0 || d < bd) { bd = d; ii = f; }
  }
  // edge axes over every face pair (faces of a tiled, of b repeated) and
  // edge pair; get_edge_support picks the best
  int best = -1;
  float best_v = 0.f, best_sd = 0.f;
  v3 best_ax = mk(0.f, 0.f, 0.f), ba1 = best_ax, ba2 = best_ax, bb1 = best_ax, bb2 = best_ax;
  for (int kp = 0; kp < 36; kp++) {
    const int fa = kp % 6, fb = kp / 6;
    for (int m = 0; m < 16; m++) {
      const int ea = m & 3, eb = m >> 2;
      const v3 a1 = A.f[fa][ea], a2 = A.f[fa][(ea + 3) & 3];
      const v3 b1 = B.f[fb][eb], b2 = B.f[fb][(eb + 3) & 3];
      v3 ax = cross(a1 - a2, b1 - b2);
      ax = ax * (dot(a1 - origin, ax) > 0.f ? 1.f : -1.f);
      bool bad = ax.x == 0.f && ax.y == 0.f && ax.z == 0.f;
      float mx = 0.f;
      for (int v = 0; v < 8; v++) {
        float t = dot(ax, A.v[v] - a1);
        mx = (v == 0 || t > mx) ? t : mx;
      }
      bad |= mx > 0.f;
      v3 dm = (a1 + (a2 - a1) * 0.5f) - (b1 + (b2 - b1) * 0.5f);
      const float aux = -dot(dm, dm);
      int sv = 0;
      float sd = 0.f;
      for (int v = 0; v < 8; v++) {
        float t = dot(ax, B.v[v] - a1);
        if (v == 0 || t < sd) { sd = t; sv = v; }
      }
      const v3 spt = B.v[sv];
      const float s1 = ((b1.x - spt.x) + (b1.y - spt.y)) + (b1.z - spt.z);
      const float s2 = ((b2.x - spt.x) + (b2.y - spt.y)) + (b2.z - spt.z);
      if (!(s1 == 0.f || s2 == 0.f)) bad = true;
      if (bad) sd = -1e6f;
      const float val = sd + aux;
      if (best < 0 || val > best_v) {
        best_v = val; best = kp * 16 + m; best_sd = sd; best_ax = ax;
        ba1 = a1; ba2 = a2; bb1 = b1; bb2 = b2;
      }
    }
  }
  const float edge_dist = best_sd;
  const bool maybe_edge = edge_dist > face_dist;
  const v3 en = pdiv3(best_ax, safe_norm(best_ax));
  const bool has_int = fmaxf(edge_dist, face_dist) < 0.f;
  // _create_sat_edge_contact: closest points with the barycentric t
  v3 da = ba2 - ba1, db = bb2 - bb1;
  float la = safe_norm(da);
  la += 1e-6f * (float)(la == 0.f);
  da = pdiv3(da, la);
  float lb = safe_norm(db);
  lb += 1e-6f * (float)(lb == 0.f);
  db = pdiv3(db, lb);
  const float hla = la * 0.5f, hlb = lb * 0.5f;
  const v3 am = ba1 + da * hla, bm = bb1 + db * hlb, tr = am - bm;
  const float dadb = dot(da, db), datr = dot(da, tr), dbtr = dot(db, tr);
  const float ota = pdiv(-datr + dadb * dbtr, (1.f - dadb * dadb) + 1e-6f);
  const float otb = dbtr + ota * dadb;
  v3 pa = am + da * clampf(ota, -hla, hla), pb = bm + db * clampf(otb, -hlb, hlb);
  {
    v3 na, nb;
    float dd1 = seg_point(ba1, ba2, pb, na);
    float dd2 = seg_point(bb1, bb2, pa, nb);
    if (dd1 < dd2) pa = na; else pb = nb;
  }
  const float ta = pdiv(ota + hla, la), tb = pdiv(otb + hlb, lb);
  const bool valid = has_int && maybe_edge && ta >= 0.f && ta <= 1.f && tb >= 0.f && tb <= 1.f;
  const float edge_pen0 = valid ? -edge_dist : -1.f;
  if (edge_pen0 > 0.f) {  // jp.cond(edge_contact.penetration[0] > 0, edge, face)
    pos = pb + (pa - pb) * 0.5f;
    n = -en;
    pen = e == 0 ? edge_pen0 : -1.f;
  } else {
    hull_manifold(ref_face, inc_faces[ii], ref_n, inc_ns[ii], use_b ? 1.f : -1.f, e, pos, n, pen);
  }
  vel = (a.vel + cross(a.ang, pos - a.pos)) - (b.vel + cross(b.ang, pos - b.pos));
}

// every contact function of row r (the item-loop kernels)
template <int F>
__device__ __forceinline__ void contact_gen_x(const Cst& c, const BlobHdr& H, int r, const RowC& R,
                                              const QP& a, const QP& b, v3& pos, v3& vel, v3& n,
                                              float& pen) {
  if constexpr ((F & F_X) != 0) {
    const int o = H.o_row + r * ROW_STRIDE;
    if (R.fn == BX_COL_HEIGHTMAP) { heightmap_contact(c, H, o, R, a, b, pos, vel, n, pen); return; }
    if (R.fn == BX_COL_CLIPPED_PLANE) { clipped_contact(c, o, R, a, b, pos, vel, n, pen); return; }
    if (R.fn == BX_COL_CAPSULE_MESH) { capsule_mesh_contact(c, o, R, a, b, pos, vel, n, pen); return; }
    if (R.fn == BX_COL_HULL_HULL) { hull_contact(c, H, o, a, b, pos, vel, n, pen); return; }
  }
  contact_gen<F>(R, a, b, pos, vel, n, pen);
}

// One/TwoWay._position_contact (colliders.py:306-377, 495-580)
// RAWL (the MULTI kernel): oar / obr carry, in x, y, z, each side's angular
// impulse before the body's quaternion product (w = 0): the body forms
// 0.5 vec_quat_mul(I L, rot) once from its rows' summed L, as the update is
// linear in L (the reference's per-row quaternions, summed, are the same)
template <int F, bool RAWL = false>
__device__ __forceinline__ float position_contact(const RowC& R, const QP& a, const QP& b, const v3& ao_pos,
                                  const q4& ao_rot, const v3& bo_pos, const q4& bo_rot, v3 cpos,
                                  v3 n, float cpen, v3& oap, q4& oar, v3& obp, q4& obr) {
  BX_IEEE_IN_CONTACT
  float sc = R.scale;
  if (is_oneway<F>(R.oneway)) {
    v3 pp = cpos, pc = cpos + n * cpen;
    v3 dx = pp - pc;
    pp = pp - a.pos;
    float c = dot(dx, n);
    v3 cr1 = cross(pp, n);
    float w1 = 1.f / R.ma + dot(cr1, mul(R.Ia, cr1));
    float dl = -c / (w1 + 1e-6f);
    float cm = c < 0.f ? 1.f : 0.f;
    v3 pv = dl * n * cm;
    // static friction
    v3 r1 = rotate(cpos - a.pos, quat_inv(a.rot));
    v3 p1bar = ao_pos + rotate(r1, ao_rot);
    v3 dp = cpos - p1bar;
    v3 dt = dp - dot(dp, n) * n;
    float c2 = cancel_norm(dt);
    v3 n2 = dt / (c2 + 1e-6f);
    cr1 = cross(pp, n2);
    w1 = 1.f / R.ma + dot(cr1, mul(R.Ia, cr1));
    float dlt = -c2 / (w1 + 0.f);
    float sm = fabsf(dlt) < fabsf(R.fric * dl) ? 1.f : 0.f;
    // the normal and friction impulses share the lever arm: one position and
    // one quaternion update for their sum (both linear in the impulse)
    pv = pv + dlt * n2 * sm * cm;
    oap = sc * (pv / R.ma);
    if constexpr (RAWL) {
      const v3 L = sc * cross(pp, pv);
      oar = q4{0.f, L.x, L.y, L.z};
    } else {
      oar = sc * (0.5f * vec_quat_mul(mul(R.Ia, cross(pp, pv)), a.rot));
    }
    obp = mk(0.f, 0.f, 0.f);
    obr = q4{0.f, 0.f, 0.f, 0.f};
    return dl * cm;
  }
  v3 pp = cpos - n * cpen / 2.f - a.pos;
  v3 pc = cpos + n * cpen / 2.f - b.pos;
  float c = -cpen;
  v3 cr1 = cross(pp, n), cr2 = cross(pc, n);
  float w1 = 1.f / R.ma + dot(cr1, mul(R.Ia, cr1));
  float w2 = 1.f / R.mb + dot(cr2, mul(R.Ib, cr2));
  float dl = -c / (w1 + w2 + 1e-6f);
  float cm = c < 0.f ? 1.f : 0.f;
  v3 pv = dl * n * cm;
  // angular impulses of the normal and friction parts (their lever arms
  // differ) add up before one quaternion product per body
  const v3 la = cross(pp, pv), lb = cross(pc, pv);
  v3 r1 = rotate(cpos - a.pos, quat_inv(a.rot));
  v3 r2 = rotate(cpos - b.pos, quat_inv(b.rot));
  v3 p1bar = ao_pos + rotate(r1, ao_rot);
  v3 p2bar = bo_pos + rotate(r2, bo_rot);
  v3 dp = (cpos - p1bar) - (cpos - p2bar);
  v3 dt = dp - dot(dp, n) * n;
  pp = cpos - a.pos;
  pc = cpos - b.pos;
  float c2 = cancel_norm(dt);
  v3 n2 = dt / (c2 + 1e-6f);
  cr1 = cross(pp, n2);
  cr2 = cross(pc, n2);
  w1 = 1.f / R.ma + dot(cr1, mul(R.Ia, cr1));
  w2 = 1.f / R.mb + dot(cr2, mul(R.Ib, cr2));
  float dlt = -c2 / (w1 + w2);
  float sm = fabsf(dlt) < fabsf(dl) ? 1.f : 0.f;
  const v3 pt = dlt * n2 * sm * cm;
  const v3 ps = pv + pt;
  oap = sc * (ps / R.ma);
  obp = sc * (-ps / R.mb);
  if constexpr (RAWL) {
    const v3 La = sc * (la + cross(pp, pt)), Lb = -sc * (lb + cross(pc, pt));
    oar = q4{0.f, La.x, La.y, La.z};
    obr = q4{0.f, Lb.x, Lb.y, Lb.z};
  } else {
    oar = sc * (0.5f * vec_quat_mul(mul(R.Ia, la + cross(pp, pt)), a.rot));
    obr = sc * (-0.5f * vec_quat_mul(mul(R.Ib, lb + cross(pc, pt)), b.rot));
  }
  return dl;
}

// One/TwoWay._velocity_contact (colliders.py:379-442, 584-658);
// (aov, aoa, aop) = qp_right_before of body a (vel, ang, pos), same for b.
template <int F>
__device__ __forceinline__ void velocity_contact(const RowC& R, float h, const QP& a, const QP& b, v3 aop,
                                 v3 aov, v3 aoa, v3 bop, v3 bov, v3 boa, v3 cpos, v3 n, float cpen,
                                 float dlam, v3& oav, v3& oaa, v3& obv, v3& oba) {
  BX_IEEE_IN_CONTACT
  v3 ra = cpos - a.pos, rb = cpos - b.pos;
  v3 rv = is_oneway<F>(R.oneway) ? a.vel + cross(a.ang, ra)
                   : (a.vel + cross(a.ang, ra)) - (b.vel + cross(b.ang, rb));
  float vn = dot(rv, n);
  v3 vt = rv - n * vn;
  float vtn = cancel_norm(vt);
  v3 vtd = vt / (1e-6f + vtn);
  float lim = R.fric * fabsf(dlam) / (2.f * h);
  float mag = fminf(lim, vtn);
  v3 dvel = -vtd * mag;
  v3 pdyn;
  if (is_oneway<F>(R.oneway)) {
    v3 aw = cross(ra, vtd);
    float w = 1.f / R.ma + dot(aw, aw);
    pdyn = dvel / (w + 1e-6f);
  } else {
    v3 a1 = cross(ra, vtd), a2 = cross(rb, vtd);
    float w1 = 1.f / R.ma + dot(a1, mul(R.Ia, a1));
    float w2 = 1.f / R.mb + dot(a2, mul(R.Ib, a2));
    pdyn = dvel / (w1 + w2 + 1e-6f);
  }
  v3 rvo = is_oneway<F>(R.oneway) ? aov + cross(aoa, cpos - aop)
                    : (aov + cross(aoa, cpos - aop)) - (bov + cross(boa, cpos - bop));
  float vno = dot(rvo, n);
  float mn = fminf(R.elas * vno, 0.f);
  v3 dvr = n * (-vn - mn);
  v3 pp = cpos - a.pos;
  v3 pc = (cpos + n * cpen) - b.pos;
  float c = cancel_norm(dvr);
  v3 n2 = dvr / (c + 1e-6f);
  v3 cr1 = cross(pp, n2);
  float w1 = 1.f / R.ma + dot(cr1, mul(R.Ia, cr1));
  float dlr;
  if (is_oneway<F>(R.oneway)) {
    dlr = c / (w1 + 1e-6f);
  } else {
    v3 cr2 = cross(pc, n2);
    float w2 = 1.f / R.mb + dot(cr2, mul(R.Ib, cr2));
    dlr = c / (w1 + w2 + 1e-6f);
  }
  float sm = cpen > 0.f ? 1.f : 0.f;
  float sink = is_oneway<F>(R.oneway) ? (vno <= -R.thr ? 1.f : 0.f) : (vno <= 0.f ? 1.f : 0.f);
  v3 pv = (dlr * n2 * sink + pdyn) * sm;
  oav = pv / R.ma;
  oaa = cross(mul(R.Ia, ra), pv);
  if (is_oneway<F>(R.oneway)) {
    obv = mk(0.f, 0.f, 0.f);
    oba = mk(0.f, 0.f, 0.f);
  } else {
    obv = -pv / R.mb;
    oba = cross(mul(R.Ib, rb), -pv);
  }
}

// One/TwoWay._contact (colliders.py:267-304, 449-493): the impulse model used
// by System.info at reset.
template <int F>
__device__ void impulse_contact(const RowC& R, const QP& a, const QP& b, v3 cpos, v3 cvel, v3 n,
                                float cpen, v3& oav, v3& oaa, v3& obv, v3& oba) {
  BX_IEEE_IN_SPRING
  v3 rpa = cpos - a.pos, rpb = cpos - b.pos;
  float bv = R.erp * cpen;
  float nv = dot(n, cvel);
  v3 x1 = cross(mul(R.Ia, cross(rpa, n)), rpa);
  float denom;
  if (is_oneway<F>(R.oneway)) {
    denom = 1.f / R.ma + dot(n, x1);
  } else {
    v3 x2 = cross(mul(R.Ib, cross(rpb, n)), rpb);
    denom = 1.f / R.ma + 1.f / R.mb + dot(n, x1 + x2);
  }
  float imp = (-1.f * (1.f + R.elas) * nv + bv) / denom;
  v3 vd = cvel - nv * n;
  float vdn = safe_norm(vd);
  float impd = fminf(vdn / denom, R.fric * imp);
  v3 dird = vd / (1e-6f + vdn);
  float an = (cpen > 0.f && nv < 0.f && imp > 0.f) ? 1.f : nan_of(cpen);
  float ad = an * (vdn > 0.01f ? 1.f : 0.f);
  v3 J = imp * n, Jd = -impd * dird;
  oav = (J / R.ma) * an + (Jd / R.ma) * ad;
  oaa = mul(R.Ia, cross(rpa, J)) * an + mul(R.Ia, cross(rpa, Jd)) * ad;
  if (is_oneway<F>(R.oneway)) {
    obv = mk(0.f, 0.f, 0.f);
    oba = mk(0.f, 0.f, 0.f);
  } else {
    v3 Jb = -imp * n, Jdb = impd * dird;
    obv = (Jb / R.mb) * an + (Jdb / R.mb) * ad;
    oba = mul(R.Ib, cross(rpb, Jb)) * an + mul(R.Ib, cross(rpb, Jdb)) * ad;
  }
}

// Torque/Angle.apply_reduced for actuator a (lane) -> aslot
template <int F, int LS = 16>
__device__ __forceinline__ void act_torque(const JointC& Jc, const ActC& A, const Env& E,
                                           const float* al, int a, bool useJL = false,
                                           JLim JL = JLim{}, const uint4* LI = nullptr,
                                           const v3* tqd = nullptr) {
  BX_IEEE_IN_JOINT
  QP p = ldqp(E.qp + Jc.bp * QP_STRIDE), cq = ldqp(E.qp + Jc.bc * QP_STRIDE);
  if (LI && is_torque<F>(A.type)) {
    // torque actuators on the lane image's limit rows: the angles
    // (axis_angle) enter only the limit cut, taken on pseudo-angles
    v3 tq;
    const float t0 = al[0] * A.strength * -1.f;
    if (is_rev<F>(Jc.type)) {
      const v3 axis = rotate(Jc.axp[0], p.rot);
      const v3 ref_p = rotate(Jc.axp[2], p.rot), ref_c = rotate(Jc.axc[2], cq.rot);
      const float pa = pseudo_angle(dot(ref_p, ref_c), dot(cross(ref_p, ref_c), axis));
      const float2 L = ld_lim_p<LS>(LI, LIM_G0);
      tq = mk(0.f, 0.f, 0.f) + axis * ((pa < L.x || pa > L.y) ? 0.f : t0);
    } else {
      // Spherical.axis_angle (joints.py:388-415): psi, theta = +-acos(cb)
      // (the pseudo-angle of (cb, +-sqrt(1 - cb^2))), phi
      // (each body's axes through its rotation matrix: the same arithmetic as
      // the spherical joint halves, which rotate one body per lane)
      const RotM Mp = rot_matrix(p.rot), Mc = rot_matrix(cq.rot);
      const v3 a1p = mrot(Mp, Jc.axp[0]), a2p = mrot(Mp, Jc.axp[1]);
      const v3 a1c = mrot(Mc, Jc.axc[0]), a2c = mrot(Mc, Jc.axc[1]), a3c = mrot(Mc, Jc.axc[2]);
      // pseudo-angles are scale-free in (x, y): lon and xz enter unnormalised,
      // (cb, sqrt(1 - cb^2)) as (x, sqrt(|xz|^2 - x^2)) with x = xz . a1p
      const v3 lon = cross(a3c, a1p);
      const v3 xz = dot(a1p, a1c) * a1c + dot(a1p, a2c) * a2c;
      const float xb = dot(xz, a1p), r2 = dot(xz, xz);
      const float sg = signf(dot(a1p, a3c));
      const float yb = r2 > 0.f ? sg * __builtin_amdgcn_sqrtf(fmaxf(r2 - xb * xb, 0.f)) : sg;
      float pa[3];
      pa[0] = pseudo_angle(dot(a2p, lon), dot(cross(a2p, lon), a1p));
      pa[1] = pseudo_angle(sg == 0.f ? 1.f : xb, yb);
      pa[2] = pseudo_angle(dot(a2c, lon), dot(cross(a2c, lon), -a3c));
      const v3 axes[3] = {a1p, a2c, a3c};
      tq = mk(0.f, 0.f, 0.f);
      float2 Lp[3];
#pragma unroll
      for (int l = 0; l < 3; l++) Lp[l] = ld_lim_p<LS>(LI, lim_group(l));
#pragma unroll
      for (int l = 0; l < 3; l++) {
        const float t = al[l] * A.strength * -1.f;
        tq = tq + axes[l] * ((pa[l] < Lp[l].x || pa[l] > Lp[l].y) ? 0.f : t);
      }
    }
    if (tqd) tq = tq + *tqd;  // + the joint's damping (FOLD)
    st_v3a(E.aslot + a * ASLOT_STRIDE, mul(Jc.Ip, tq));
    st_v3a(E.aslot + (E.nK + a) * ASLOT_STRIDE, -1.f * mul(Jc.Ic, tq));
    return;
  }
  if (useJL && is_rev<F>(Jc.type) && is_torque<F>(A.type)) {
    // a revolute torque actuator needs its hinge angle only for the limit
    // cut: the test on pseudo-angles (no atan2)
    const v3 axis = rotate(Jc.axp[0], p.rot);
    const v3 ref_p = rotate(Jc.axp[2], p.rot), ref_c = rotate(Jc.axc[2], cq.rot);
    const float pa = pseudo_angle(dot(ref_p, ref_c), dot(cross(ref_p, ref_c), axis));
    float t = al[0] * A.strength * -1.f;
    if (pa < JL.plo) t = 0.f;
    if (pa > JL.phi) t = 0.f;
    const v3 tq = mk(0.f, 0.f, 0.f) + axis * t;
    st_v3a(E.aslot + a * ASLOT_STRIDE, mul(Jc.Ip, tq));
    st_v3a(E.aslot + (E.nK + a) * ASLOT_STRIDE, -1.f * mul(Jc.Ic, tq));
    return;
  }
  v3 axes[3];
  float ang[3];
  int dof = axis_angle<F>(Jc, p, cq, axes, ang);
  v3 tq = mk(0.f, 0.f, 0.f);
#pragma unroll
  for (int l = 0; l < 3; l++) {
    if (l < dof) {
      float t;
      if (is_torque<F>(A.type)) {
        t = al[l] * A.strength * -1.f;
        if (ang[l] < Jc.lim[2 * l]) t = 0.f;
        if (ang[l] > Jc.lim[2 * l + 1]) t = 0.f;
      } else {
        float tgt = clampf(deg_to_rad(al[l]), Jc.lim[2 * l], Jc.lim[2 * l + 1]);
        t = (tgt - ang[l]) * A.strength;
      }
      tq = tq + axes[l] * t;
    }
  }
  float sgp = is_torque<F>(A.type) ? 1.f : -1.f;
  st_v3a(E.aslot + a * ASLOT_STRIDE, sgp * mul(Jc.Ip, tq));
  st_v3a(E.aslot + (E.nK + a) * ASLOT_STRIDE, -sgp * mul(Jc.Ic, tq));
}


// ---------------------------------------------------------------------------
// joint halves (F_JH, SINGLE mode at 16 lanes with <= 8 revolute joints, Ant):
// lane j works the parent side of joint j and lane j + 8 its child side. The
// two sides of a revolute constraint are the same arithmetic on each body's
// own frame (world anchor, lever arm, effective mass, impulse, rotation
// update), so one instruction stream serves both halves and exchanges the few
// cross terms with the partner lane by a DPP row rotation; the shared scalar
// work (constraint norm, limit angle, angle-update direction) is computed
// redundantly. Each lane then writes its side's slot. Halves the per-lane
// instruction count of the joint and actuator phases (Ant leaves lanes 8-15
// idle there otherwise).
// ---------------------------------------------------------------------------
enum { F_JH = 128 };

// the partner half's value: lane ^ 8 within the env's 16-lane row
// (bound_ctrl set: a row rotation has no invalid source lane, so the `old`
// operand is dead and needs no zeroing v_mov before each exchange)
__device__ __forceinline__ float xh(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x128, 0xF, 0xF, true));
}
__device__ __forceinline__ v3 xh3(v3 v) { return mk(xh(v.x), xh(v.y), xh(v.z)); }
__device__ __forceinline__ v3 sel3(bool s, v3 a, v3 b) {
  return mk(s ? a.x : b.x, s ? a.y : b.y, s ? a.z : b.z);
}

// Contact halves (SINGLE mode, F_R2G's two-way capsule-capsule slot): row k's
// a side on lane k, its b side on lane k + 8 of the env's 16 (partner xh,
// lane ^ 8). Both lanes hold the row's contact (contact_gen of the same words:
// the same bits); each forms its own body's terms of TwoWay._position_contact
// / _velocity_contact and trades them with the partner, so the shared values
// (the effective-mass sums, the rest-pose drift, the relative velocities)
// come out as the one-lane functions above form them, bit for bit, and each
// lane returns only its own side's impulse. The two lanes run at once where
// one lane ran both sides in turn.
__device__ __forceinline__ float pick_a(bool sb, float own, float other) { return sb ? other : own; }
__device__ __forceinline__ float pick_b(bool sb, float own, float other) { return sb ? own : other; }

template <int F>
__device__ __forceinline__ float position_contact_half(const RowC& R, const QP& o, const v3& oo_pos,
                                                       const q4& oo_rot, v3 cpos, v3 n, float cpen,
                                                       bool sb, v3& op, q4& orr) {
  BX_IEEE_IN_CONTACT
  const float sc = R.scale;
  const float m = sb ? R.mb : R.ma;
  const v3 I = sb ? R.Ib : R.Ia;
  const v3 hn = n * cpen / 2.f;
  const v3 pq = (sb ? cpos + hn : cpos - hn) - o.pos;  // a: pp, b: pc
  const float c = -cpen;
  v3 cr = cross(pq, n);
  float w = 1.f / m + dot(cr, mul(I, cr));
  float wp = xh(w);
  const float dl = -c / (pick_a(sb, w, wp) + pick_b(sb, w, wp) + 1e-6f);
  const float cm = c < 0.f ? 1.f : 0.f;
  const v3 pv = dl * n * cm;
  const v3 l0 = cross(pq, pv);  // a: la, b: lb
  const v3 r = rotate(cpos - o.pos, quat_inv(o.rot));
  const v3 pbar = oo_pos + rotate(r, oo_rot);
  const v3 pbp = xh3(pbar);
  const v3 p1bar = sel3(sb, pbp, pbar), p2bar = sel3(sb, pbar, pbp);
  const v3 dp = (cpos - p1bar) - (cpos - p2bar);
  const v3 dt = dp - dot(dp, n) * n;
  const v3 pr = cpos - o.pos;  // a: pp, b: pc (the friction lever)
  const float c2 = cancel_norm(dt);
  const v3 n2 = dt / (c2 + 1e-6f);
  cr = cross(pr, n2);
  w = 1.f / m + dot(cr, mul(I, cr));
  wp = xh(w);
  const float dlt = -c2 / (pick_a(sb, w, wp) + pick_b(sb, w, wp));
  const float sm = fabsf(dlt) < fabsf(dl) ? 1.f : 0.f;
  const v3 pt = dlt * n2 * sm * cm;
  const v3 ps = pv + pt;
  op = sb ? sc * (-ps / m) : sc * (ps / m);
  orr = sb ? sc * (-0.5f * vec_quat_mul(mul(I, l0 + cross(pr, pt)), o.rot))
           : sc * (0.5f * vec_quat_mul(mul(I, l0 + cross(pr, pt)), o.rot));
  return dl;
}

template <int F>
__device__ __forceinline__ void velocity_contact_half(const RowC& R, float h, const QP& o, v3 oop, v3 oov,
                                                      v3 ooa, v3 cpos, v3 n, float cpen, float dlam,
                                                      bool sb, v3& ov, v3& oa) {
  BX_IEEE_IN_CONTACT
  const float m = sb ? R.mb : R.ma;
  const v3 I = sb ? R.Ib : R.Ia;
  const v3 ro = cpos - o.pos;  // a: ra, b: rb
  const v3 t = o.vel + cross(o.ang, ro);
  const v3 tp = xh3(t);
  const v3 rv = sel3(sb, tp, t) - sel3(sb, t, tp);
  float vn = dot(rv, n);
  v3 vt = rv - n * vn;
  float vtn = cancel_norm(vt);
  v3 vtd = vt / (1e-6f + vtn);
  float lim = R.fric * fabsf(dlam) / (2.f * h);
  float mag = fminf(lim, vtn);
  v3 dvel = -vtd * mag;
  const v3 a1 = cross(ro, vtd);
  float w = 1.f / m + dot(a1, mul(I, a1));
  float wp = xh(w);
  const v3 pdyn = dvel / (pick_a(sb, w, wp) + pick_b(sb, w, wp) + 1e-6f);
  const v3 to = oov + cross(ooa, cpos - oop);
  const v3 top = xh3(to);
  const v3 rvo = sel3(sb, top, to) - sel3(sb, to, top);
  float vno = dot(rvo, n);
  float mn = fminf(R.elas * vno, 0.f);
  v3 dvr = n * (-vn - mn);
  const v3 pq = (sb ? cpos + n * cpen : cpos) - o.pos;  // a: pp, b: pc
  float c = cancel_norm(dvr);
  v3 n2 = dvr / (c + 1e-6f);
  const v3 cr = cross(pq, n2);
  w = 1.f / m + dot(cr, mul(I, cr));
  wp = xh(w);
  const float dlr = c / (pick_a(sb, w, wp) + pick_b(sb, w, wp) + 1e-6f);
  float smk = cpen > 0.f ? 1.f : 0.f;
  float sink = vno <= 0.f ? 1.f : 0.f;
  v3 pv = (dlr * n2 * sink + pdyn) * smk;
  ov = sb ? -pv / m : pv / m;
  oa = cross(mul(I, ro), sb ? -pv : pv);
}



// Revolute.apply_reduced (joints.py:79-100, 154-195, 270-309), one side: o is
// this side's body (parent on lanes 0-7, child on 8-15); returns its dp, dq
__device__ __forceinline__ void joint_apply_half(const JointC& J, const JLim& JL, const JSide& S,
                                                 bool child, const QP& o, v3& dpo, q4& dro) {
  const float sg = S.sg;
  const v3 I = S.I;
  const float m = S.m;
  // this side's three vectors through one rotation matrix
  const RotM Mo = rot_matrix(o.rot);
  // positional constraint
  v3 wo = o.pos + mrot(Mo, S.off);
  v3 ro = wo - o.pos;
  v3 wt = xh3(wo);
  // the parent's anchor minus the child's on both halves, bit for bit (IEEE
  // a - b is exactly -(b - a)); the effective masses add commutatively
  v3 dx = sg * (wo - wt);
  float cc = cancel_norm(dx);
  v3 n = dx / (cc + 1e-6f);
  v3 cr = cross(ro, n);
  float wm = 1.f / m + dot(cr, mul(I, cr));
  float wp = xh(wm);
  float dl = -cc / (wm + wp + 1e-6f);
  v3 pv = dl * n;
  dpo = J.sp * ((sg * pv) / m);
  // the two angular constraints (axis alignment, limited hinge angle)
  v3 u0 = mrot(Mo, S.ax0);
  v3 u2 = mrot(Mo, S.ax2);
  v3 t0 = xh3(u0), t2 = xh3(u2);
  // the parent lane computes dq1's impulse, the child lane dq2's, and they
  // trade them: each lane forms only its own correction, from its own
  // vectors in the parent / child order that lane sees them (parent: u =
  // the parent's, t = the child's; child: the reverse)
  v3 dq1 = cross(u0, t0);                               // valid on the parent lane
  v3 dq2 = cross(hinge_turn(t0, t2, u2, JL), u2);       // valid on the child lane
  const v3 pm = angle_impulse(J, sel3(child, dq2, dq1));
  const v3 po = xh3(pm);
  // the side's rotation update is linear in the angular impulse: the
  // position constraint's and both angle constraints' add up before the one
  // quaternion product (joints.py:150-152, 190-195)
  const v3 P = J.sp * cross(ro, pv) + J.sa * (pm + po);
  dro = (sg * 0.5f) * vec_quat_mul(mul(I, P), o.rot);
}

// Actuator.apply_reduced (actuators.py:52-112) for a revolute joint, one side
template <int F>
__device__ __forceinline__ void act_torque_half(const JointC& Jc, const JLim& JL, const JSide& S,
                                                const ActC& A, const Env& E, const float* al, int a,
                                                bool child, const q4& ro, const v3* tqd = nullptr) {
  v3 u0 = rotate(S.ax0, ro);
  v3 u2 = rotate(S.ax2, ro);
  v3 t0 = xh3(u0), t2 = xh3(u2);
  v3 axis = sel3(child, t0, u0);
  const v3 ref_p = sel3(child, t2, u2), ref_c = sel3(child, u2, t2);
  float t;
  if (is_torque<F>(A.type)) {
    // the torque is cut outside the limits: the hinge angle's limit test on
    // pseudo-angles (no atan2)
    const float pa = pseudo_angle(dot(ref_p, ref_c), dot(cross(ref_p, ref_c), axis));
    t = al[0] * A.strength * -1.f;
    if (pa < JL.plo) t = 0.f;
    if (pa > JL.phi) t = 0.f;
  } else {
    float ang = signed_angle(axis, ref_p, ref_c);
    float tgt = clampf(deg_to_rad(al[0]), Jc.lim[0], Jc.lim[1]);
    t = (tgt - ang) * A.strength;
  }
  v3 tq = mk(0.f, 0.f, 0.f) + axis * t;
  float sgp = is_torque<F>(A.type) ? 1.f : -1.f;
  // parent: sgp * Ip tq, child: -sgp * Ic tq (the side's sign times its inertia)
  float* slot = E.aslot + (child ? E.nK + a : a) * ASLOT_STRIDE;
  if (tqd) st_v3a(slot, S.sg * mul(S.I, sgp * tq + *tqd));  // + the joint's damping (FOLD)
  else st_v3a(slot, (sgp * S.sg) * mul(S.I, tq));
}

// ---------------------------------------------------------------------------
// per-env LDS carving
// ---------------------------------------------------------------------------
// every LDS region starts 16-byte aligned (offsets are multiples of 4 words,
// env blocks of 64 words): telling the compiler lets it use ds_read_b128 /
// ds_write_b128 (and b64/b96) instead of pairs of 4-byte accesses
__device__ __forceinline__ float* al16(float* p) {
  return reinterpret_cast<float*>(__builtin_assume_aligned(p, 16));
}

__device__ __forceinline__ Env carve(float* base, const BlobHdr& H, bool multi = false) {
  Env E;
  E.qp = al16(base + H.l_qp);
  E.prev = al16(base + H.l_prev);
  E.rb = al16(base + H.l_rb);
  E.jslot = al16(base + H.l_jslot);
  E.aslot = al16(base + H.l_aslot);
  E.rowd = al16(base + H.l_rowd);
  E.cslot = al16(base + H.l_cslot);
  E.acc = al16(base + H.l_acc);
  E.ang = al16(base + H.l_ang);
  E.red = al16(base + H.l_red);
  E.ract = reinterpret_cast<int*>(base + H.l_ract);
  E.alist = reinterpret_cast<int*>(base + H.l_alist);
  E.nJ = H.J;
  E.nK = H.K;
  E.nR = H.R;
  E.xact = al16(base + H.l_xact);
  E.arow = al16(base + H.l_arow);
  E.nnl = al16(base + H.l_nnl);
  E.jlim = reinterpret_cast<uint4*>(al16(base + H.l_jlim));
  if (multi) {
    // MULTI: 6-word contact slots, 8-word task partials; no row-data region (the
    // row's contact stays in its lane's registers); the task partials double
    // as NearNeighbors scratch before the substeps
    E.rowd = nullptr;
    E.cslot = al16(base + H.l_mslot);
    E.acc = E.cslot;  // the Info accumulators, written after the last pass
    E.tslot = al16(base + H.l_tslot);
    E.nearl = reinterpret_cast<uint16_t*>(base + H.l_near);
    E.nnl = E.tslot;  // NearNeighbors' lists, before the first task phase
    E.nearc = reinterpret_cast<int*>(base + H.l_cnt);
    E.sidx = reinterpret_cast<uint16_t*>(base + H.l_sidx);
    E.cbuf = al16(base + H.l_cbuf);
    E.ract = reinterpret_cast<int*>(E.cbuf);  // NearNeighbors' ranks, before the first pass
    E.bimg = reinterpret_cast<uint32_t*>(base + H.l_bimg);
    E.cen = reinterpret_cast<uint4*>(al16(base + H.l_cen));
    E.mat = E.cen + 2 * H.n_cen;
    E.bod = E.mat + H.n_mat;
    E.sstride = MSLOT_STRIDE;
    E.nd = E.tslot;
    E.nds = 1;
  } else {
    E.tslot = nullptr;
    E.sstride = SLOT_STRIDE;
    E.nd = E.rowd + 8;  // rowd word 8 is free until the first position pass
    E.nds = ROWD_STRIDE;
  }
  return E;
}

// Phase boundary inside one env block. Every kernel that calls this runs
// 64-thread workgroups = ONE wavefront, and a wavefront's LDS instructions
// execute in issue order, so a lane's ds_read issued after another lane's
// ds_write sees it without draining lgkmcnt. Only the compiler must not move
// or forward memory accesses across the boundary.
__device__ __forceinline__ void sync() { asm volatile("" ::: "memory"); }
// pbd_step_single's phase boundaries (A/B knob -DBX_NOSYNC_SINGLE: none; the
// compiler's own alias analysis then keeps every LDS store before the loads
// that may read it, the gather indices being runtime values, and the machine
// scheduler may overlap one phase's tail with the next's independent work,
// which an inline-asm boundary forbids)
__device__ __forceinline__ void phase_sync() {
#if !defined(BX_NOSYNC_SINGLE)
  sync();
#endif
}
// An env spread over L > 64 threads (large scenes: 128 or 256 threads = 2-4
// waves of one workgroup, one env per workgroup) needs a real workgroup
// barrier at each phase boundary; within one wave the compiler fence above.
template <int L>
__device__ __forceinline__ void esync() {
  if constexpr (L > 64) __syncthreads(); else sync();
}

// a culled row's slots: no update, not counted (the item-loop kernels; the
// MULTI kernel's NearNeighbors zeroes its 6-word slots from its row tables)
__device__ __forceinline__ void zero_row_slots(const Cst& c, const BlobHdr& H, const Env& E, int r) {
  float* sa = E.cslot + r * E.sstride;
  float* sb = E.cslot + (E.nR + r) * E.sstride;
  for (int k = 0; k < 8; k++) { sa[k] = 0.f; sb[k] = 0.f; }
}

// NearNeighbors.update (colliders.py:71-85) for every culled group, from the
// env's current qp: candidate-centre distance of each allowed cell, then the
// `cutoff` nearest cells get ranks 0.. (top_k of -dist; equal distances to the
// lower flat index = row index, as jax.lax.top_k). Ranks go to E.ract.
// min of v over the env's lanes of one wave: W = 16 (a DPP row), 32 or 64
// (the rows combined through readlane), in every lane of the segment. Every
// lane of the wave must be active. (A one-pass 64-bit variant with row
// broadcasts measured slower: 31.7k vs 28.7k cycles of picks per step.)
template <int W>
__device__ __forceinline__ unsigned seg_min_u32(unsigned v) {
  v = min(v, (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, 0x128, 0xF, 0xF, true));  // row_ror:8
  v = min(v, (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, 0x124, 0xF, 0xF, true));  // row_ror:4
  v = min(v, (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, 0x122, 0xF, 0xF, true));  // row_ror:2
  v = min(v, (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, 0x121, 0xF, 0xF, true));  // row_ror:1
  if constexpr (W == 16) {
    return v;
  } else {
    const unsigned a = (unsigned)__builtin_amdgcn_readlane((int)v, 0);
    const unsigned b = (unsigned)__builtin_amdgcn_readlane((int)v, 16);
    const unsigned c2 = (unsigned)__builtin_amdgcn_readlane((int)v, 32);
    const unsigned d = (unsigned)__builtin_amdgcn_readlane((int)v, 48);
    if constexpr (W == 32) return (threadIdx.x & 32) ? min(c2, d) : min(a, b);
    return min(min(a, b), min(c2, d));
  }
}

// the sum over each 16-lane row (one env at 16 lanes) in every lane of the
// row: a row_ror butterfly (every lane of the wave must be active)
__device__ __forceinline__ float row_sum16(float v) {
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x128, 0xF, 0xF, true));
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x124, 0xF, 0xF, true));
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x122, 0xF, 0xF, true));
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x121, 0xF, 0xF, true));
  return v;
}

// v of lane ^ d within the wave (d = 1, 2, 4, 8 by DPP: quad permutes, row
// shifts, the row rotation; 16, 32 by ds_bpermute)
__device__ __forceinline__ unsigned lane_xor(unsigned v, int d) {
  switch (d) {
    case 1: return (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, 0xB1, 0xF, 0xF, true);   // quad_perm 1,0,3,2
    case 2: return (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, 0x4E, 0xF, 0xF, true);   // quad_perm 2,3,0,1
    case 4: {
      const unsigned up = (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, 0x104, 0xF, 0xF, true);  // row_shl:4
      const unsigned dn = (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xF, 0xF, true);  // row_shr:4
      return (threadIdx.x & 4) ? dn : up;
    }
    case 8: return (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, 0x128, 0xF, 0xF, true);  // row_ror:8
    default: return (unsigned)__shfl_xor((int)v, d, 64);
  }
}

// a candidate cell's selection key: (distance bits, row); distances are >= 0,
// so their bit patterns order like the floats; a masked cell's sim is -inf,
// its key (+inf's bits) sorts after every finite distance, ties in row =
// flat order as jax.lax.top_k keeps them
__device__ __forceinline__ unsigned long long nn_key(const Cst& c, const BlobHdr& H, const Env& E,
                                                     int r) {
  const int o = H.o_row + r * ROW_STRIDE;
  unsigned d = 0x7F800000u;
  if (!c.i(o + R_NNMASK)) {
    const int ba = c.i(o + R_A), bb = c.i(o + R_B);
    QP a = ldqp(E.qp + ba * QP_STRIDE), b = ldqp(E.qp + bb * QP_STRIDE);
    v3 pa = a.pos + rotate(c.f3(o + R_APOS), a.rot);
    v3 pb = b.pos + rotate(c.f3(o + R_BPOS), b.rot);
    d = __float_as_uint(norm(pb - pa));
  }
  return ((unsigned long long)d << 32) | (unsigned)r;
}

// NearNeighbors.update (colliders.py:71-85) for every culled group, from the
// env's current qp: candidate-centre distance of each allowed cell, then the
// `cutoff` nearest cells get ranks 0.. (top_k of -dist; equal distances to the
// lower flat index = row index, as jax.lax.top_k). Ranks go to E.ract, the
// selected rows in Info order to E.alist.
//
// Each lane holds its (<= NK) candidates' keys sorted in registers; the
// env's part in each wave picks its `cutoff` smallest keys by DPP minima
// (no LDS, no barrier per pick); with one wave per env those are the ranks,
// with several, each wave's sorted list goes to LDS and every listed key
// counts the smaller keys of the other lists (its rank in the union).
// Groups with more than NK candidates per lane take the serial pick.
// MULTI: the collidables' centres (E.cen: n_cen (body, offset | end, radius)
// records) placed in the world from the env's current qp, after the bodies'
// table (the caller syncs)
template <int L>
__device__ __forceinline__ void place_centres(const BlobHdr& H, const Env& E, int lane) {
  uint4* cw = E.bod + H.N;
  for (int k = lane; k < H.n_cen; k += L) {
    const uint4 cc = E.cen[2 * k];
    const float* qb = E.qp + (int)cc.x * QP_STRIDE;
    const v3 p = ld3(qb) + rotate(mk(__uint_as_float(cc.y), __uint_as_float(cc.z),
                                     __uint_as_float(cc.w)), ld_rot(qb));
    cw[k] = make_uint4(__float_as_uint(p.x), __float_as_uint(p.y), __float_as_uint(p.z), 0u);
  }
}
// a row's collidable-centre distance from the placed centres (nn_key's and
// the broad phase's, same bits)
__device__ __forceinline__ float centre_dist(const Env& E, const BlobHdr& H, unsigned pair) {
  const uint4* cw = E.bod + H.N;
  const uint4 a4 = cw[pair & 0xFFFFu], b4 = cw[pair >> 16];
  const v3 ca = mk(__uint_as_float(a4.x), __uint_as_float(a4.y), __uint_as_float(a4.z));
  const v3 cb = mk(__uint_as_float(b4.x), __uint_as_float(b4.y), __uint_as_float(b4.z));
  return norm(cb - ca);
}

// the same squared (the broad phase compares it with its squared reach)
__device__ __forceinline__ float centre_dist2(const Env& E, const BlobHdr& H, unsigned pair) {
  const uint4* cw = E.bod + H.N;
  const uint4 a4 = cw[pair & 0xFFFFu], b4 = cw[pair >> 16];
  const v3 d = mk(__uint_as_float(b4.x), __uint_as_float(b4.y), __uint_as_float(b4.z)) -
               mk(__uint_as_float(a4.x), __uint_as_float(a4.y), __uint_as_float(a4.z));
  return dot(d, d);
}

// MULTI: a row's bounds words (BI_*): its collidable pair as centre_dist
// takes it, its flags (BIF_*), its squared reach, its Info index
__device__ __forceinline__ unsigned bi_pair(uint32_t w0) {
  return (w0 & 0xFFu) | ((w0 & 0xFF00u) << 8);
}
__device__ __forceinline__ uint32_t bi_flags(uint32_t w0) { return w0 >> 16; }
__device__ __forceinline__ float bi_reach2(uint32_t w1) {
  return (float)__builtin_bit_cast(_Float16, (unsigned short)(w1 & 0xFFFFu));
}

// MULTI: contact row r's record from the LDS tables (its flags / b slot, its
// two collidables, their bodies' masses and inverse inertias, its
// material): the words the row image held, with no L2 read
__device__ __forceinline__ RowC row_from_lds(const Env& E, int r) {
  const uint32_t w0 = E.bimg[r * BI_WORDS + BI_W0];
  const uint4 g0 = make_uint4(bi_pair(w0), 0u, bi_flags(w0), 0u);
  const uint4 a0 = E.cen[2 * (g0.x & 0xFFFFu)], a1 = E.cen[2 * (g0.x & 0xFFFFu) + 1];
  const uint4 b0 = E.cen[2 * (g0.x >> 16)], b1 = E.cen[2 * (g0.x >> 16) + 1];
  const uint4 mt = E.mat[(g0.z >> BIF_MAT_SHIFT) & 0xFFu];
  RowC x;
  x.group = 0;  // (no MULTI pass reads the group)
  x.a = (int)a0.x;
  x.b = (int)b0.x;
  x.fn = (int)((g0.z >> BIF_FN_SHIFT) & 0xFu);
  x.oneway = (g0.z & BIF_OW) ? 1 : 0;
  x.a_pos = mk(__uint_as_float(a0.y), __uint_as_float(a0.z), __uint_as_float(a0.w));
  x.a_end = mk(__uint_as_float(a1.x), __uint_as_float(a1.y), __uint_as_float(a1.z));
  x.a_rad = __uint_as_float(a1.w);
  x.b_pos = mk(__uint_as_float(b0.y), __uint_as_float(b0.z), __uint_as_float(b0.w));
  x.b_end = mk(__uint_as_float(b1.x), __uint_as_float(b1.y), __uint_as_float(b1.z));
  x.b_rad = __uint_as_float(b1.w);
  x.fric = __uint_as_float(mt.x);
  x.elas = __uint_as_float(mt.y);
  x.scale = __uint_as_float(mt.z);
  x.thr = __uint_as_float(mt.w);
  const uint4 ba = E.bod[x.a], bb = E.bod[x.b];
  x.ma = __uint_as_float(ba.x);
  x.mb = __uint_as_float(bb.x);
  x.Ia = mk(__uint_as_float(ba.y), __uint_as_float(ba.z), __uint_as_float(ba.w));
  x.Ib = mk(__uint_as_float(bb.y), __uint_as_float(bb.z), __uint_as_float(bb.w));
  return x;
}

#ifdef BX_MSTAMPS
// (diagnostic: the MULTI stamps build splits the picks' phases into slots
// 12-14 of the caller's accumulators)
#define BX_NSTAMP(k)                                                               \
  do {                                                                             \
    if (nsa) {                                                                     \
      __builtin_amdgcn_sched_barrier(0);                                           \
      unsigned long long _t;                                                       \
      asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(_t)::"memory");   \
      __builtin_amdgcn_sched_barrier(0);                                           \
      nsa[k] += _t - *nsl;                                                         \
      *nsl = _t;                                                                   \
    }                                                                              \
  } while (0)
#else
#define BX_NSTAMP(k) do {} while (0)
#endif
// MT (the MULTI kernel): each row's group flags, Info index and centre pair
// from the LDS-staged bounds (E.bimg), the keys' distances from the centres
// placed this step (place_centres, before the call): no dependent L2 reads
// (always inlined: a call would take the caller's header by reference and
// put the whole struct in scratch, reloaded in every phase of the MULTI loop)
template <int L, bool MT = false, int NK = 4>
__device__ __forceinline__ void nn_select(const Cst& c, const BlobHdr& H, const Env& E, int lane,
                          unsigned long long* nsa = nullptr, unsigned long long* nsl = nullptr) {
  // Pairs rows are always active (rank 0) at their fixed Info index; culled
  // rows start unselected with empty (zero, uncounted) slots
  if constexpr (MT) {
    // (the MULTI kernel: a culled row gets no compact index, so its slots
    // are never read)
    for (int r = lane; r < H.R; r += L) {
      const uint32_t fl = bi_flags(E.bimg[r * BI_WORDS + BI_W0]);
      if (fl & BIF_CULL) {
        E.ract[r] = -1;
      } else {
        E.ract[r] = 0;
        E.alist[E.bimg[r * BI_WORDS + BI_W1] >> 16] = r;
      }
    }
  } else
  for (int r = lane; r < H.R; r += L) {
    const int og = H.o_group + c.i(H.o_row + r * ROW_STRIDE + R_GROUP) * GROUP_STRIDE;
    if (c.i(og + G_CUT)) {
      E.ract[r] = -1;
      zero_row_slots(c, H, E, r);
    } else {
      E.ract[r] = 0;
      E.alist[c.i(og + G_INFO) + r - c.i(og + G_R0)] = r;
    }
  }
  esync<L>();
  BX_NSTAMP(14);
  constexpr int W = L < 64 ? L : 64;  // the env's lanes in one wave
  constexpr int NW = L / W;           // the env's waves
  // NK: candidates per lane held in registers (4; the 128-thread MULTI
  // kernel 8, so a wave still holds a culled group of up to 8 x 128 rows)
  static_assert(NK == 4 || NK == 8, "4 or 8 keys per lane");
  const int wl = lane % W;            // lane within the env's part of its wave
  const int wv = lane / W;            // the env's wave
  for (int g = 0; g < H.G; g++) {
    const int og = H.o_group + g * GROUP_STRIDE;
    const int cut = c.i(og + G_CUT);
    if (cut == 0) continue;
    const int r0 = c.i(og + G_R0), r1 = c.i(og + G_R1), info = c.i(og + G_INFO);
    if (r1 - r0 <= NK * L && (NW == 1 || 2 * NW * cut <= H.nnl_words)) {
      unsigned long long k[NK];
#pragma unroll
      for (int i = 0; i < NK; i++) {
        const int r = r0 + lane + i * L;
        if constexpr (MT) {
          if (r < r1) {
            const uint32_t w0 = E.bimg[r * BI_WORDS + BI_W0];
            const unsigned d = (bi_flags(w0) & BIF_MASK) ? 0x7F800000u
                                                         : __float_as_uint(centre_dist(E, H, bi_pair(w0)));
            k[i] = ((unsigned long long)d << 32) | (unsigned)r;
          } else {
            k[i] = ~0ull;
          }
        } else {
          k[i] = r < r1 ? nn_key(c, H, E, r) : ~0ull;
        }
      }
      // sorting network on the lane's keys
      auto cs = [](unsigned long long& a, unsigned long long& b) {
        const unsigned long long lo = a < b ? a : b, hi = a < b ? b : a;
        a = lo;
        b = hi;
      };
      if constexpr (NK == 4) {
        cs(k[0], k[1]); cs(k[2], k[3]); cs(k[0], k[2]); cs(k[1], k[3]); cs(k[1], k[2]);
      } else {
        // Batcher's odd-even merge sort of 8 (19 compare-exchanges)
        cs(k[0], k[1]); cs(k[2], k[3]); cs(k[4], k[5]); cs(k[6], k[7]);
        cs(k[0], k[2]); cs(k[1], k[3]); cs(k[4], k[6]); cs(k[5], k[7]);
        cs(k[1], k[2]); cs(k[5], k[6]);
        cs(k[0], k[4]); cs(k[1], k[5]); cs(k[2], k[6]); cs(k[3], k[7]);
        cs(k[2], k[4]); cs(k[3], k[5]);
        cs(k[1], k[2]); cs(k[3], k[4]); cs(k[5], k[6]);
      }
      BX_NSTAMP(12);
      unsigned long long* lst = reinterpret_cast<unsigned long long*>(E.nnl);
      if constexpr (NW > 1) {
        // each wave's NK x 64 keys sorted ascending by a bitonic network
        // (element NK wl + q in lane wl's k[q]): the lane's sorted NK are
        // the size-NK blocks (odd lanes' reversed: descending), then per block
        // size the lane-exchange strides (>= NK elements: lane ^ stride / NK,
        // two 32-bit lane swizzles per key) and the in-lane strides NK / 2 ..
        // 1. The union's order is the picks' (distance, then row: the 64-bit
        // key); its first `cut` keys are the wave's list.
        static_assert(NW == 1 || W == 64, "bitonic lists: NK keys x 64 lanes");
        if (wl & 1) {
#pragma unroll
          for (int q = 0; q < NK / 2; q++) {
            const unsigned long long t = k[q];
            k[q] = k[NK - 1 - q];
            k[NK - 1 - q] = t;
          }
        }
        auto ced = [](unsigned long long& a, unsigned long long& b, bool up) {
          const bool sw = up ? (b < a) : (a < b);
          const unsigned long long x = a;
          a = sw ? b : a;
          b = sw ? x : b;
        };
#pragma unroll
        for (int size = 2 * NK; size <= 64 * NK; size <<= 1) {
          const bool up = ((wl * NK) & size) == 0;
#pragma unroll
          for (int d = size / (2 * NK); d >= 1; d >>= 1) {
            const bool keep_min = ((wl & d) == 0) == up;
#pragma unroll
            for (int q = 0; q < NK; q++) {
              const unsigned lo = lane_xor((unsigned)k[q], d);
              const unsigned hi = lane_xor((unsigned)(k[q] >> 32), d);
              const unsigned long long o = ((unsigned long long)hi << 32) | lo;
              k[q] = keep_min ? (o < k[q] ? o : k[q]) : (o < k[q] ? k[q] : o);
            }
          }
#pragma unroll
          for (int st = NK / 2; st >= 1; st >>= 1)
#pragma unroll
            for (int q = 0; q < NK; q++)
              if ((q & st) == 0) ced(k[q], k[q + st], up);
        }
#pragma unroll
        for (int q = 0; q < NK; q++)
          if (NK * wl + q < cut) lst[wv * cut + NK * wl + q] = k[q];
        // (a cut past the wave's NK x 64 keys: the rest of its list is empty)
        for (int i = NK * W + wl; i < cut; i += W) lst[wv * cut + i] = ~0ull;
      } else
      for (int kk = 0; kk < cut; kk++) {
        const unsigned long long cur = k[0];
        const unsigned hi = (unsigned)(cur >> 32), lo = (unsigned)cur;
        // the segment's smallest key: its distance, then its row among equals
        const unsigned dmin = seg_min_u32<W>(hi);
        const unsigned rmin = seg_min_u32<W>(hi == dmin ? lo : ~0u);
        const bool own = cur != ~0ull && hi == dmin && lo == rmin;
        if (own) {
          // the picked key leaves the lane's sorted registers
#pragma unroll
          for (int q = 0; q + 1 < NK; q++) k[q] = k[q + 1];
          k[NK - 1] = ~0ull;
          if constexpr (NW == 1) {
            E.ract[(int)lo] = kk;
            E.alist[info + kk] = (int)lo;
          }
        }
        if constexpr (NW > 1) {
          if (wl == 0) lst[wv * cut + kk] = ((unsigned long long)dmin << 32) | rmin;
        }
      }
      if constexpr (NW > 1) {
        esync<L>();
        BX_NSTAMP(13);
        for (int t = lane; t < NW * cut; t += L) {
          const int w = t / cut, i = t % cut;
          const unsigned long long key = lst[t];
          if (key == ~0ull) continue;
          // + the smaller keys of each other (sorted) list: branch-free lower
          // bounds, the lists' probes issued together
          int base[NW];
#pragma unroll
          for (int w2 = 0; w2 < NW; w2++) base[w2] = w2 * cut;
          for (int len = cut; len > 1;) {
            const int half = len >> 1;
#pragma unroll
            for (int w2 = 0; w2 < NW; w2++)
              base[w2] = lst[base[w2] + half - 1] < key ? base[w2] + half : base[w2];
            len -= half;
          }
          int rank = i;
#pragma unroll
          for (int w2 = 0; w2 < NW; w2++)
            if (w2 != w) rank += base[w2] - w2 * cut + (lst[base[w2]] < key ? 1 : 0);
          if (rank < cut) {
            E.ract[(int)(unsigned)key] = rank;
            E.alist[info + rank] = (int)(unsigned)key;
          }
        }
      }
      esync<L>();
      continue;
    }
    // serial pick: candidate-centre distance of every cell, once (E.nd:
    // scratch until the position pass of the first substep), then `cut`
    // minima over the env's lanes
    for (int r = r0 + lane; r < r1; r += L) {
      const unsigned long long key = nn_key(c, H, E, r);
      E.nd[r * E.nds] = __uint_as_float((unsigned)(key >> 32));
    }
    esync<L>();
    for (int k = 0; k < cut; k++) {
      unsigned long long best = ~0ull;
      for (int r = r0 + lane; r < r1; r += L) {
        if (E.ract[r] >= 0) continue;
        const float d = E.nd[r * E.nds];
        unsigned long long key = ((unsigned long long)__float_as_uint(d) << 32) | (unsigned)r;
        best = key < best ? key : best;
      }
      // minimum over the env's L lanes (aligned L-lane segment of the wave)
#pragma unroll
      for (int off = W / 2; off > 0; off >>= 1) {
        unsigned lo = __shfl_xor((unsigned)best, off, W);
        unsigned hi = __shfl_xor((unsigned)(best >> 32), off, W);
        unsigned long long o2 = ((unsigned long long)hi << 32) | lo;
        best = o2 < best ? o2 : best;
      }
      if constexpr (L > 64) {
        // then over the env's waves: each wave's minimum through LDS
        // (red words 40.. hold one 64-bit key per wave)
        unsigned long long* wk = reinterpret_cast<unsigned long long*>(E.red + 40);
        if ((lane & 63) == 0) wk[lane >> 6] = best;
        __syncthreads();
#pragma unroll
        for (int w = 0; w < L / 64; w++) best = wk[w] < best ? wk[w] : best;
      }
      const int r = (int)(best & 0xFFFFFFFFu);
      if (((r - r0) % L) == lane) {
        E.ract[r] = k;
        E.alist[info + k] = r;
      }
      esync<L>();
    }
  }
}

__device__ __forceinline__ bool row_active(const BlobHdr& H, const Env& E, int r) {
  return H.n_nn == 0 || E.ract[r] >= 0;
}

// Info contact index of row r (system.py:36-43), -1 when culled this step
__device__ __forceinline__ int row_info(const Cst& c, const BlobHdr& H, const Env& E, int r) {
  const int og = H.o_group + c.i(H.o_row + r * ROW_STRIDE + R_GROUP) * GROUP_STRIDE;
  if (c.i(og + G_CUT) == 0) return c.i(og + G_INFO) + r - c.i(og + G_R0);
  const int k = E.ract[r];
  return k < 0 ? -1 : c.i(og + G_INFO) + k;
}

// the zero slots that padded gather-list entries point at
__device__ __forceinline__ void zero_slots(const Env& E, const BlobHdr& H, int lane) {
  if (lane < SLOT_STRIDE) {
    E.jslot[2 * H.J * SLOT_STRIDE + lane] = 0.f;
    if (lane < E.sstride) E.cslot[(E.tslot ? H.m_zero : 2 * H.R) * E.sstride + lane] = 0.f;
    if (lane < ASLOT_STRIDE) E.aslot[2 * H.K * ASLOT_STRIDE + lane] = 0.f;
    if (E.tslot && lane < TSLOT_STRIDE) E.tslot[H.T * TSLOT_STRIDE + lane] = 0.f;
  }
}

// global <-> LDS QP through strided field views
__device__ __forceinline__ void load_qp_regs(const bx_qp& q, int64_t e, int b, float* s) {
  const float* p = q.pos.ptr + e * q.pos.env_stride + b * q.pos.body_stride;
  const float* r = q.rot.ptr + e * q.rot.env_stride + b * q.rot.body_stride;
  const float* v = q.vel.ptr + e * q.vel.env_stride + b * q.vel.body_stride;
  const float* a = q.ang.ptr + e * q.ang.env_stride + b * q.ang.body_stride;
  s[0] = p[0]; s[1] = p[1]; s[2] = p[2];
  s[3] = r[0]; s[4] = r[1]; s[5] = r[2]; s[6] = r[3];
  s[7] = v[0]; s[8] = v[1]; s[9] = v[2];
  s[10] = a[0]; s[11] = a[1]; s[12] = a[2];
}
__device__ __forceinline__ void load_qp_global(const bx_qp& q, int64_t e, int b, float* s) {
  const float* p = q.pos.ptr + e * q.pos.env_stride + b * q.pos.body_stride;
  const float* r = q.rot.ptr + e * q.rot.env_stride + b * q.rot.body_stride;
  const float* v = q.vel.ptr + e * q.vel.env_stride + b * q.vel.body_stride;
  const float* a = q.ang.ptr + e * q.ang.env_stride + b * q.ang.body_stride;
  s[0] = p[0]; s[1] = p[1]; s[2] = p[2];
  s[3] = r[0]; s[4] = r[1]; s[5] = r[2]; s[6] = r[3];
  s[7] = v[0]; s[8] = v[1]; s[9] = v[2];
  s[10] = a[0]; s[11] = a[1]; s[12] = a[2];
}
__device__ __forceinline__ void store_qp_global(const bx_qp& q, int64_t e, int b, const float* s) {
  float* p = q.pos.ptr + e * q.pos.env_stride + b * q.pos.body_stride;
  float* r = q.rot.ptr + e * q.rot.env_stride + b * q.rot.body_stride;
  float* v = q.vel.ptr + e * q.vel.env_stride + b * q.vel.body_stride;
  float* a = q.ang.ptr + e * q.ang.env_stride + b * q.ang.body_stride;
  p[0] = s[0]; p[1] = s[1]; p[2] = s[2];
  r[0] = s[3]; r[1] = s[4]; r[2] = s[5]; r[3] = s[6];
  v[0] = s[7]; v[1] = s[8]; v[2] = s[9];
  a[0] = s[10]; a[1] = s[11]; a[2] = s[12];
}

// ---------------------------------------------------------------------------
// the PBD step of one env (system.py:254-325), all L lanes of the env
// ---------------------------------------------------------------------------
template <int L, int F>
__device__ void pbd_step(const Cst& c, const BlobHdr& H, const Env& E, int lane, bool valid,
                         const float* act, int aw) {
  const int N = H.N, J = H.J, K = H.K, Rn = H.R;
  const float h = H.h;
  for (int b = lane; b < N; b += L) {
    float* acc = E.acc + b * ACC_STRIDE;
    for (int k = 0; k < 9; k++) acc[k] = 0.f;
  }
  // cull.update once per step, before the substeps (system.py:320-321)
  if (H.n_nn) nn_select<L>(c, H, E, lane);
  for (int it = 0; it < H.substeps / 2; it++) {
    for (int sub = 0; sub < 2; sub++) {
      // qprev = qp
      for (int b = lane; b < N; b += L) {
        const float* s = E.qp + b * QP_STRIDE;
        float* d = E.prev + b * PREV_STRIDE;
        for (int k = 0; k < 7; k++) d[k] = s[k];
      }
      // actuators (actuators.py:52-112) and joint damping (joints.py:103-128)
      for (int a = lane; a < K; a += L) {
        ActC A = load_act(c, H, a);
        JointC Jc = load_joint(c, H, A.joint);
        float al[3];
#pragma unroll
        for (int l = 0; l < 3; l++) {
          int ai = A.idx[l];
          al[l] = valid ? act[take_idx(ai, aw)] * (ai >= 0 ? 1.f : 0.f) : 0.f;
        }
        act_torque<F>(Jc, A, E, al, a);
      }
      for (int j = lane; j < J; j += L) {
        int o = H.o_joint + j * JOINT_STRIDE;
        int bp = c.i(o + J_BP), bc = c.i(o + J_BC);
        float damp = c.f(o + J_DAMP);
        v3 Ip = c.f3(H.o_body + bp * BODY_STRIDE + BODY_I);
        v3 Ic = c.f3(H.o_body + bc * BODY_STRIDE + BODY_I);
        v3 tq = -1.f * damp * (ld3(E.qp + bp * QP_STRIDE + 10) - ld3(E.qp + bc * QP_STRIDE + 10));
        st3(E.jslot + j * SLOT_STRIDE, mul(Ip, tq));
        st3(E.jslot + (E.nJ + j) * SLOT_STRIDE, -1.f * mul(Ic, tq));
      }
      esync<L>();
      // Euler.update(acc) + Euler.kinetic (integrators.py:50-93)
      for (int b = lane; b < N; b += L) {
        BodyC B = load_body(c, H, b);
        v3 dpa = mk(0.f, 0.f, 0.f), dpj = mk(0.f, 0.f, 0.f);
        for (int i = c.i(H.o_al_off + b), e = c.i(H.o_al_off + b + 1); i < e; i++)
          dpa = dpa + ld3(E.aslot + c.i(H.o_al + i) * ASLOT_STRIDE);
        for (int i = c.i(H.o_jl_off + b), e = c.i(H.o_jl_off + b + 1); i < e; i++)
          dpj = dpj + ld3(E.jslot + c.i(H.o_jl + i) * SLOT_STRIDE);
        QP q = ldqp(E.qp + b * QP_STRIDE);
        v3 fv, fa;  // dp_f (forces.py), acc_p = (dp_a + dp_f) + dp_j (system.py:268-271)
        body_forces(c, H, b, act, aw, valid, fv, fa);
        v3 vel = H.vexp * q.vel;
        vel = vel + (fv + mk(H.gx, H.gy, H.gz)) * h;
        vel = mul(vel, B.pm);
        v3 ang = H.aexp * q.ang;
        ang = ang + ((dpa + fa) + dpj) * h;
        ang = mul(ang, B.rm);
        q.vel = vel;
        q.ang = ang;
        q.pos = q.pos + mul(q.vel * h, B.pm);
        v3 am = mul(q.ang, B.rm);
        q4 hq = (q4{0.f, am.x, am.y, am.z} * 0.5f) * h;
        q4 r = q.rot + quat_mul(hq, q.rot);
        q.rot = qnormalize(r);
        stqp(E.qp + b * QP_STRIDE, q);
        if (sub == 1) st3(E.acc + b * ACC_STRIDE + ACC_DPA, dpa);
      }
      esync<L>();
      // Joint.apply (joints.py:79-100)
      for (int j = lane; j < J; j += L) {
        JointC Jc = load_joint(c, H, j);
        QP p = ldqp(E.qp + Jc.bp * QP_STRIDE), q = ldqp(E.qp + Jc.bc * QP_STRIDE);
        v3 dpp, dcp;
        q4 dpr, dcr;
        joint_apply<F>(Jc, p, q, dpp, dpr, dcp, dcr, false, JLim{}, nullptr,
                       c.w + H.o_joint + j * JOINT_STRIDE);
        float* sp = E.jslot + j * SLOT_STRIDE;
        float* sc = E.jslot + (E.nJ + j) * SLOT_STRIDE;
        st3(sp, dpp); st4(sp + 3, dpr);
        st3(sc, dcp); st4(sc + 3, dcr);
      }
      esync<L>();
      // Euler.update(pos) (+ velocity_projection on the first substep)
      for (int b = lane; b < N; b += L) {
        BodyC B = load_body(c, H, b);
        v3 dp = mk(0.f, 0.f, 0.f);
        q4 dr{0.f, 0.f, 0.f, 0.f};
        for (int i = c.i(H.o_jl_off + b), e = c.i(H.o_jl_off + b + 1); i < e; i++) {
          const float* s = E.jslot + c.i(H.o_jl + i) * SLOT_STRIDE;
          dp = dp + ld3(s);
          dr = dr + ld4(s + 3);
        }
        float* s = E.qp + b * QP_STRIDE;
        QP q = ldqp(s);
        q.pos = q.pos + mul(dp, B.pm);
        q.rot = q4{q.rot.w + dr.w * B.qm.w, q.rot.x + dr.x * B.qm.x, q.rot.y + dr.y * B.qm.y,
                   q.rot.z + dr.z * B.qm.z};
        if (sub == 0) {
          // Euler.velocity_projection (integrators.py:122-146)
          const float* pv = E.prev + b * PREV_STRIDE;
          v3 ppos = ld3(pv);
          q4 prot = ld4(pv + 3);
          q4 nr = qnormalize(q.rot);
          q.vel = mul((q.pos - ppos) / h, B.pm);
          q4 dq = quat_mul(nr, quat_inv(prot));
          v3 a = 2.f * mk(dq.x, dq.y, dq.z) / h;
          float scl = dq.w >= 0.f ? 1.f : -1.f;
          q.ang = mul(mul(scl * B.rm, a), B.rm);
          q.rot = nr;
        }
        stqp(s, q);
      }
      esync<L>();
    }
    // ---- collisions on the second substep (system.py:288-313)
    // Collider.position_apply (colliders.py:198-240)
    // with culling: only the step's active rows (culled slots stay zero)
    for (int i = lane; i < (H.n_nn ? H.info_rows : Rn); i += L) {
      const int r = H.n_nn ? E.alist[i] : i;
      RowC R = load_row(c, H, r);
      QP a = ldqp(E.qp + R.a * QP_STRIDE), b = ldqp(E.qp + R.b * QP_STRIDE);
      v3 cpos, cvel, n;
      float pen;
      contact_gen_x<F>(c, H, r, R, a, b, cpos, cvel, n, pen);
      const float* pa = E.prev + R.a * PREV_STRIDE;
      const float* pb = E.prev + R.b * PREV_STRIDE;
      v3 oap, obp;
      q4 oar, obr;
      float dl = position_contact<F>(R, a, b, ld3(pa), ld4(pa + 3), ld3(pb), ld4(pb + 3), cpos, n, pen,
                                  oap, oar, obp, obr);
      if (is_nan(pen)) {
        // a NaN contact's impulses are NaN on both sides (the reference's
        // masked products, colliders.py:332-333: NaN * 0)
        const float pz = nan_of(pen);
        oap = obp = mk(pz, pz, pz);
        oar = obr = q4{pz, pz, pz, pz};
        dl = pz;
      }
      float* rd = E.rowd + r * ROWD_STRIDE;
      st3(rd, cpos); st3(rd + 3, n); rd[6] = pen; rd[7] = dl;
      float* sa = E.cslot + r * SLOT_STRIDE;
      float* sb = E.cslot + (E.nR + r) * SLOT_STRIDE;
      st3(sa, oap); st4(sa + 3, oar);
      sa[7] = nonzero3(oap);
      st3(sb, obp); st4(sb + 3, obr);
      sb[7] = nonzero3(obp);
    }
    esync<L>();
    for (int b = lane; b < N; b += L) {
      BodyC B = load_body(c, H, b);
      v3 dp = mk(0.f, 0.f, 0.f);
      q4 dr{0.f, 0.f, 0.f, 0.f};
      int i = c.i(H.o_cl_off + b), e = c.i(H.o_cl_off + b + 1);
      while (i < e) {
        int g = c.i(H.o_cl + i) >> 24;
        v3 gp = mk(0.f, 0.f, 0.f);
        q4 gr{0.f, 0.f, 0.f, 0.f};
        float cnt = 0.f;
        for (; i < e && (c.i(H.o_cl + i) >> 24) == g; i++) {
          const float* s = E.cslot + (c.i(H.o_cl + i) & 0xFFFFFF) * SLOT_STRIDE;
          gp = gp + ld3(s);
          gr = gr + ld4(s + 3);
          cnt += s[7];
        }
        float d = 1e-6f + cnt;
        dp = dp + gp / d;
        dr = dr + q4{gr.w / d, gr.x / d, gr.y / d, gr.z / d};
      }
      float* s = E.qp + b * QP_STRIDE;
      QP q = ldqp(s);
      q.pos = q.pos + mul(dp, B.pm);
      q.rot = q4{q.rot.w + dr.w * B.qm.w, q.rot.x + dr.x * B.qm.x, q.rot.y + dr.y * B.qm.y,
                 q.rot.z + dr.z * B.qm.z};
      // qp_right_before, then velocity_projection
      float* rb = E.rb + b * RB_STRIDE;
      st3(rb, q.pos); st3(rb + 3, q.vel); st3(rb + 6, q.ang);
      const float* pv = E.prev + b * PREV_STRIDE;
      v3 ppos = ld3(pv);
      q4 prot = ld4(pv + 3);
      q4 nr = qnormalize(q.rot);
      q.vel = mul((q.pos - ppos) / h, B.pm);
      q4 dq = quat_mul(nr, quat_inv(prot));
      v3 a = 2.f * mk(dq.x, dq.y, dq.z) / h;
      float scl = dq.w >= 0.f ? 1.f : -1.f;
      q.ang = mul(mul(scl * B.rm, a), B.rm);
      q.rot = nr;
      stqp(s, q);
    }
    esync<L>();
    // Collider.velocity_apply (colliders.py:155-196)
    for (int i = lane; i < (H.n_nn ? H.info_rows : Rn); i += L) {
      const int r = H.n_nn ? E.alist[i] : i;
      RowC R = load_row(c, H, r);
      QP a = ldqp(E.qp + R.a * QP_STRIDE), b = ldqp(E.qp + R.b * QP_STRIDE);
      const float* ra = E.rb + R.a * RB_STRIDE;
      const float* rbb = E.rb + R.b * RB_STRIDE;
      const float* rd = E.rowd + r * ROWD_STRIDE;
      v3 oav, oaa, obv, oba;
      velocity_contact<F>(R, h, a, b, ld3(ra), ld3(ra + 3), ld3(ra + 6), ld3(rbb), ld3(rbb + 3),
                       ld3(rbb + 6), ld3(rd), ld3(rd + 3), rd[6], rd[7], oav, oaa, obv, oba);
      if (is_nan(rd[6])) {
        const float pz = nan_of(rd[6]);
        oav = oaa = obv = oba = mk(pz, pz, pz);
      }
      float* sa = E.cslot + r * SLOT_STRIDE;
      float* sb = E.cslot + (E.nR + r) * SLOT_STRIDE;
      st3(sa, oav); st3(sa + 3, oaa);
      sa[7] = nonzero3(oav);
      st3(sb, obv); st3(sb + 3, oba);
      sb[7] = nonzero3(obv);
    }
    esync<L>();
    for (int b = lane; b < N; b += L) {
      BodyC B = load_body(c, H, b);
      v3 dv = mk(0.f, 0.f, 0.f), da = mk(0.f, 0.f, 0.f);
      int i = c.i(H.o_cl_off + b), e = c.i(H.o_cl_off + b + 1);
      while (i < e) {
        int g = c.i(H.o_cl + i) >> 24;
        v3 gv = mk(0.f, 0.f, 0.f), ga = mk(0.f, 0.f, 0.f);
        float cnt = 0.f;
        for (; i < e && (c.i(H.o_cl + i) >> 24) == g; i++) {
          const float* s = E.cslot + (c.i(H.o_cl + i) & 0xFFFFFF) * SLOT_STRIDE;
          gv = gv + ld3(s);
          ga = ga + ld3(s + 3);
          cnt += s[7];
        }
        float d = 1e-6f + cnt;
        dv = dv + gv / d;
        da = da + ga / d;
      }
      float* s = E.qp + b * QP_STRIDE;
      v3 vel = mul(ld3(s + 7) + dv, B.pm);
      v3 ang = mul(ld3(s + 10) + da, B.rm);
      st3(s + 7, vel);
      st3(s + 10, ang);
      float* acc = E.acc + b * ACC_STRIDE;
      st3(acc + ACC_ICV, ld3(acc + ACC_ICV) + dv);
      st3(acc + ACC_ICA, ld3(acc + ACC_ICA) + da);
      st3(acc + ACC_IAA, ld3(acc + ACC_IAA) + ld3(acc + ACC_DPA));
    }
    esync<L>();
  }
}

// Collider.apply over the step's active rows (colliders.py:116-153): impulse
// contacts into the row slots (vel 0..2, ang 3..5, any() flag 7) and the row
// data (contact pos, normal, penetration) for Info
template <int L, int F>
__device__ void impulse_rows(const Cst& c, const BlobHdr& H, const Env& E, int lane) {
  for (int i = lane; i < (H.n_nn ? H.info_rows : H.R); i += L) {
    const int r = H.n_nn ? E.alist[i] : i;
    RowC R = load_row(c, H, r);
    QP a = ldqp(E.qp + R.a * QP_STRIDE), b = ldqp(E.qp + R.b * QP_STRIDE);
    v3 cpos, cvel, n;
    float pen;
    contact_gen_x<F>(c, H, r, R, a, b, cpos, cvel, n, pen);
    v3 oav, oaa, obv, oba;
    impulse_contact<F>(R, a, b, cpos, cvel, n, pen, oav, oaa, obv, oba);
    float* rd = E.rowd + r * ROWD_STRIDE;
    st3(rd, cpos); st3(rd + 3, n); rd[6] = pen;
    float* sa = E.cslot + r * SLOT_STRIDE;
    float* sb = E.cslot + (E.nR + r) * SLOT_STRIDE;
    st3(sa, oav); st3(sa + 3, oaa);
    sa[7] = nonzero3(oav);
    st3(sb, obv); st3(sb + 3, oba);
    sb[7] = nonzero3(obv);
  }
}

// per-body (vel, ang) update of the rows' slots: each collider group summed
// and divided by (eps + #non-zero rows), groups added in order
__device__ __forceinline__ void contact_reduce(const Cst& c, const BlobHdr& H, const Env& E, int b,
                                               float eps, v3& dv, v3& da) {
  BX_IEEE_IN_SPRING
  dv = mk(0.f, 0.f, 0.f);
  da = mk(0.f, 0.f, 0.f);
  int i = c.i(H.o_cl_off + b), e = c.i(H.o_cl_off + b + 1);
  while (i < e) {
    int g = c.i(H.o_cl + i) >> 24;
    v3 gv = mk(0.f, 0.f, 0.f), ga = mk(0.f, 0.f, 0.f);
    float cnt = 0.f;
    for (; i < e && (c.i(H.o_cl + i) >> 24) == g; i++) {
      const float* s = E.cslot + (c.i(H.o_cl + i) & 0xFFFFFF) * SLOT_STRIDE;
      gv = gv + ld3(s);
      ga = ga + ld3(s + 3);
      cnt += s[7];
    }
    float d = eps + cnt;
    dv = dv + gv / d;
    da = da + ga / d;
  }
}

// ---------------------------------------------------------------------------
// System._spring_step (system.py:342-375), all L lanes of the env: per
// substep Euler.kinetic, spring joints + actuators + forces at the
// acceleration level, then Collider.apply at the velocity level. Info:
// contact += dp_c, joint += dp_j (in E.rb words 0..5), actuator += dp_a.
// ---------------------------------------------------------------------------
template <int L, int F>
__device__ void spring_step(const Cst& c, const BlobHdr& H, const Env& E, int lane, bool valid,
                            const float* act, int aw) {
  const int N = H.N, J = H.J, K = H.K;
  const float h = H.h;
  for (int b = lane; b < N; b += L) {
    float* acc = E.acc + b * ACC_STRIDE;
    for (int k = 0; k < 9; k++) acc[k] = 0.f;
    float* ij = E.rb + b * RB_STRIDE;
    for (int k = 0; k < 6; k++) ij[k] = 0.f;
  }
  if (H.n_nn) nn_select<L>(c, H, E, lane);
  for (int sub = 0; sub < H.substeps; sub++) {
    // Euler.kinetic (integrators.py:50-68)
    for (int b = lane; b < N; b += L) {
      BodyC B = load_body(c, H, b);
      QP q = ldqp(E.qp + b * QP_STRIDE);
      q.pos = q.pos + mul(q.vel * h, B.pm);
      v3 am = mul(q.ang, B.rm);
      q4 hq = (q4{0.f, am.x, am.y, am.z} * 0.5f) * h;
      q4 r = q.rot + quat_mul(hq, q.rot);
      q.rot = qnormalize(r);
      stqp(E.qp + b * QP_STRIDE, q);
    }
    esync<L>();
    // spring Joint.apply (spring_joints.py:89-113) -> joint slots (vel, ang)
    for (int j = lane; j < J; j += L) {
      JointC Jc = load_joint(c, H, j);
      SpringC S = load_spring(c, H, j);
      QP p = ldqp(E.qp + Jc.bp * QP_STRIDE), q = ldqp(E.qp + Jc.bc * QP_STRIDE);
      v3 dvp, dap, dvc, dac;
      spring_joint_apply(Jc, S, p, q, dvp, dap, dvc, dac);
      float* sp = E.jslot + j * SLOT_STRIDE;
      float* sc = E.jslot + (E.nJ + j) * SLOT_STRIDE;
      st3(sp, dvp); st3(sp + 3, dap);
      st3(sc, dvc); st3(sc + 3, dac);
    }
    // actuators (actuators.py:52-112) -> actuator slots
    for (int a = lane; a < K; a += L) {
      ActC A = load_act(c, H, a);
      JointC Jc = load_joint(c, H, A.joint);
      float al[3];
#pragma unroll
      for (int l = 0; l < 3; l++) {
        int ai = A.idx[l];
        al[l] = valid ? act[take_idx(ai, aw)] * (ai >= 0 ? 1.f : 0.f) : 0.f;
      }
      act_torque<F>(Jc, A, E, al, a);
    }
    esync<L>();
    // Euler.update(acc_p = dp_j + dp_a + dp_f) (integrators.py:85-93, system.py:353-357)
    for (int b = lane; b < N; b += L) {
      BodyC B = load_body(c, H, b);
      v3 jv = mk(0.f, 0.f, 0.f), ja = mk(0.f, 0.f, 0.f), dpa = mk(0.f, 0.f, 0.f);
      for (int i = c.i(H.o_jl_off + b), e = c.i(H.o_jl_off + b + 1); i < e; i++) {
        const float* s = E.jslot + c.i(H.o_jl + i) * SLOT_STRIDE;
        jv = jv + ld3(s);
        ja = ja + ld3(s + 3);
      }
      for (int i = c.i(H.o_al_off + b), e = c.i(H.o_al_off + b + 1); i < e; i++)
        dpa = dpa + ld3(E.aslot + c.i(H.o_al + i) * ASLOT_STRIDE);
      v3 fv, fa;
      body_forces(c, H, b, act, aw, valid, fv, fa);
      QP q = ldqp(E.qp + b * QP_STRIDE);
      v3 vel = H.vexp * q.vel;
      vel = vel + ((jv + fv) + mk(H.gx, H.gy, H.gz)) * h;
      q.vel = mul(vel, B.pm);
      v3 ang = H.aexp * q.ang;
      ang = ang + ((ja + dpa) + fa) * h;
      q.ang = mul(ang, B.rm);
      stqp(E.qp + b * QP_STRIDE, q);
      float* ij = E.rb + b * RB_STRIDE;
      st3(ij, ld3(ij) + jv);
      st3(ij + 3, ld3(ij + 3) + ja);
      float* acc = E.acc + b * ACC_STRIDE;
      st3(acc + ACC_IAA, ld3(acc + ACC_IAA) + dpa);
    }
    esync<L>();
    // Collider.apply (colliders.py:116-153), then Euler.update(vel_p = dp_c)
    impulse_rows<L, F>(c, H, E, lane);
    esync<L>();
    for (int b = lane; b < N; b += L) {
      BodyC B = load_body(c, H, b);
      v3 dv, da;
      contact_reduce(c, H, E, b, 1e-8f, dv, da);
      float* s = E.qp + b * QP_STRIDE;
      st3(s + 7, mul(ld3(s + 7) + dv, B.pm));
      st3(s + 10, mul(ld3(s + 10) + da, B.rm));
      float* acc = E.acc + b * ACC_STRIDE;
      st3(acc + ACC_ICV, ld3(acc + ACC_ICV) + dv);
      st3(acc + ACC_ICA, ld3(acc + ACC_ICA) + da);
    }
    esync<L>();
  }
}

// ---------------------------------------------------------------------------
// SINGLE mode: every lane owns at most one body, joint, actuator and contact
// row of its env (N, J, K, R <= L) and every per-body gather list fits MAXG.
// All constants and gather lists are hoisted into registers once per launch;
// the lane's own body state stays in registers across the substep loop and
// LDS carries only what other lanes read. No global loads inside the loop.
// ---------------------------------------------------------------------------
constexpr int MAXG = 8;

// A body's gather list, padded to M entries with the index of a zero slot so
// every gather is M unconditional LDS reads issued back-to-back (one wait).
template <int M>
struct GList {
  int e[M];
};

template <int M>
__device__ __forceinline__ GList<M> load_glist(const Cst& c, int o_off, int o_l, int b, bool has,
                                               int zero_entry) {
  GList<M> g;
  int s = c.i(o_off + b);
  int n = has ? c.i(o_off + b + 1) - s : 0;
#pragma unroll
  for (int k = 0; k < M; k++) g.e[k] = k < n ? c.i(o_l + s + k) : zero_entry;
  return g;
}

template <int M, int MC = M>
struct Hoist {
  bool hasB, hasJ, hasA, hasR, hasR2;
  bool own;   // the lane's body counts in per-body sums (JB: one copy per body)
  int r1, r2;  // the rows R and R2 (F_R2: from the lane image; else r1 = lane)
  BodyC B;
  JointC J;
  JLim JL;
  JSide S;
  ActC A;
  RowC R, R2;  // R2: F_R2's second row
  GList<M> jl, al;
  GList<MC> cl;
};

// The lane's hoisted constants from the blob's lane image (pbd_layout.h
// LI_*): every load independent and unconditional, so the whole set costs one
// L2 round trip (the records' own layout needs three dependent ones: list
// offsets -> entries, joint / row -> the bodies it references).
// JH (joint halves): lanes j and j + 8 of an env's 16 both hold joint j and
// actuator j. JB (JH, the Ant / HalfCheetah env kernels): the lane's body is
// its side's (parent of joint j on lane j, child on lane j + 8), a copy per
// side lane
template <int M, bool JH, bool R2 = false, int MC = M, bool JB = false>
__device__ __forceinline__ void load_hoist(const uint32_t* img, const BlobHdr& H, int lane,
                                           Hoist<M, MC>& X) {
  static_assert(!JB || (JH && MC <= 8), "JB: joint halves, <= 8 contact entries");
  const int jx = JH ? (lane & 7) : lane;
  X.hasB = JB ? jx < H.J : lane < H.N;
  X.hasJ = jx < H.J;
  X.hasA = jx < H.K;
  X.hasR = lane < H.R;
  X.hasR2 = false;
  X.r1 = lane;
  X.r2 = -1;
  // (img: the lane image, blob + H.o_lane; the env kernels take it from
  // their arguments, so these loads need not wait for the header)
  const uint4* im = reinterpret_cast<const uint4*>(img) + lane;
  uint32_t w[LANE_W];
  auto grab = [&](int o, int n) {
#pragma unroll
    for (int k = 0; k < n; k += 4) {
      const uint4 v = im[((o + k) / 4) * LANE_IMG_LANES];
      w[o + k] = v.x; w[o + k + 1] = v.y; w[o + k + 2] = v.z; w[o + k + 3] = v.w;
    }
  };
  constexpr int OJ = JH ? LI_JOINT_H : LI_JOINT, OA = JH ? LI_ACT_H : LI_ACT;
  constexpr int OB = JB ? LI_BODY_J : LI_BODY, OJL = JB ? LI_JL_J : LI_JL,
                OAL = JB ? LI_AL_J : LI_AL, OCL = JB ? LI_CL_J : LI_CL;
  grab(OB, 16);
  grab(OJ, 48);
  grab(OA, 8);
  grab(LI_ROW, 32);
  if constexpr (R2) {
    grab(LI_ROW2, 32);
    grab(LI_RIDX, 4);
  }
  grab(OJL, M);
  grab(OAL, M);
  grab(OCL, MC < 8 ? MC : 8);
  if constexpr (MC > 8) grab(LI_CL2, 8);
  constexpr int OL = JH ? LI_JLIM_H : LI_JLIM;
  grab(OL, 8);
  if constexpr (JH) grab(LI_SIDE_H, 16);
  auto f = [&](int i) { return __uint_as_float(w[i]); };
  auto f3 = [&](int i) { return mk(f(i), f(i + 1), f(i + 2)); };
  auto n = [&](int i) { return (int)w[i]; };
  X.B.mass = f(OB);
  X.B.I = f3(OB + 1);
  X.B.pm = f3(OB + 4);
  X.B.rm = f3(OB + 7);
  X.B.qm = q4{f(OB + 10), f(OB + 11), f(OB + 12), f(OB + 13)};
  JointC& J = X.J;
  J.type = n(OJ + LJ_TYPE);
  J.bp = n(OJ + LJ_BP);
  J.bc = n(OJ + LJ_BC);
  J.free = n(OJ + LJ_FREE);
  J.angle_off = n(OJ + LJ_AOFF);
  J.n_angles = n(OJ + LJ_NANG);
  J.dof = n(OJ + LJ_DOF);
  J.damping = f(OJ + LJ_DAMP);
  J.sp = f(OJ + LJ_SP);
  J.sa = f(OJ + LJ_SA);
  J.off_p = f3(OJ + LJ_OFFP);
  J.off_c = f3(OJ + LJ_OFFC);
#pragma unroll
  for (int k = 0; k < 3; k++) {
    J.axp[k] = f3(OJ + LJ_AXP + 3 * k);
    J.axc[k] = f3(OJ + LJ_AXC + 3 * k);
  }
#pragma unroll
  for (int k = 0; k < 6; k++) J.lim[k] = f(OJ + LJ_LIM + k);
  J.mp = f(OJ + LJ_MP);
  J.mc = f(OJ + LJ_MC);
  J.Ip = f3(OJ + LJ_IP);
  J.Ic = f3(OJ + LJ_IC);
  X.A.type = n(OA + LA_TYPE);
  X.A.joint = n(OA + LA_JOINT);
#pragma unroll
  for (int k = 0; k < 3; k++) X.A.idx[k] = n(OA + LA_IDX + k);
  X.A.strength = f(OA + LA_STR);
  auto row = [&](int o, RowC& R) {
    R.group = n(o + LR_GROUP);
    R.a = n(o + LR_A);
    R.b = n(o + LR_B);
    R.fn = n(o + LR_FN);
    R.oneway = n(o + LR_OW);
    R.a_pos = f3(o + LR_APOS);
    R.a_end = f3(o + LR_AEND);
    R.a_rad = f(o + LR_ARAD);
    R.b_pos = f3(o + LR_BPOS);
    R.b_end = f3(o + LR_BEND);
    R.b_rad = f(o + LR_BRAD);
    R.fric = f(o + LR_FRIC);
    R.elas = f(o + LR_ELAS);
    R.scale = f(o + LR_SCALE);
    R.thr = f(o + LR_THR);
    R.erp = f(o + LR_ERP);
    R.ma = f(o + LR_MA);
    R.mb = f(o + LR_MB);
    R.Ia = f3(o + LR_IA);
    R.Ib = f3(o + LR_IB);
  };
  row(LI_ROW, X.R);
  if constexpr (R2) {
    row(LI_ROW2, X.R2);
    X.r1 = n(LI_RIDX);
    X.r2 = n(LI_RIDX + 1);
    X.hasR = X.r1 >= 0;
    X.hasR2 = X.r2 >= 0;
  }
  X.JL = JLim{f(OL + LL_PLO), f(OL + LL_PHI), f(OL + LL_CLO), f(OL + LL_SLO), f(OL + LL_CHI),
               f(OL + LL_SHI)};
  if constexpr (JH) {
    X.S.off = f3(LI_SIDE_H + LS_OFF);
    X.S.ax0 = f3(LI_SIDE_H + LS_AX0);
    X.S.ax2 = f3(LI_SIDE_H + LS_AX2);
    X.S.I = f3(LI_SIDE_H + LS_I);
    X.S.m = f(LI_SIDE_H + LS_M);
    X.S.sg = f(LI_SIDE_H + LS_SG);
    X.S.body = n(LI_SIDE_H + LS_BODY);
  }
  X.own = JB ? (X.hasB && n(LI_SIDE_H + LS_OWN) != 0) : X.hasB;
#pragma unroll
  for (int k = 0; k < M; k++) {
    X.jl.e[k] = n(OJL + k);
    X.al.e[k] = n(OAL + k);
  }
#pragma unroll
  for (int k = 0; k < MC; k++) X.cl.e[k] = n(k < 8 ? OCL + k : LI_CL2 + k - 8);
}

// the spherical SINGLE kernels' limit rows into LDS, once per launch (see
// ld_lim): 6 independent 16-byte loads per lane from the lane image
template <int L, int F>
__device__ __forceinline__ void stage_lim(const uint32_t* img, const BlobHdr& H, const Env& E,
                                          int lane) {
  if constexpr ((F & F_SPH) != 0) {
    const uint4* im = reinterpret_cast<const uint4*>(img) + lane;
    constexpr int G[LIM_SLOTS] = {LI_JLIM / 4, LI_JLIM / 4 + 1, LI_JLIM12 / 4, LI_JLIM12 / 4 + 1,
                                  LI_JLIM12 / 4 + 2, LI_JLIM12 / 4 + 3};
#pragma unroll
    for (int k = 0; k < LIM_SLOTS; k++) E.jlim[k * L + lane] = im[G[k] * LANE_IMG_LANES];
  }
}

template <int M>
__device__ __forceinline__ v3 gsum3(const GList<M>& g, const float* base, int stride) {
  v3 s = mk(0.f, 0.f, 0.f);
#pragma unroll
  for (int k = 0; k < M; k++) s = s + ld_v3a(base + g.e[k] * stride);
  return s;
}

// per-group normalised contact sums  sum_g (sum of rows) / (eps + count), for
// bodies whose rows come from at most two collider groups (checked on the
// host); groups keep the reference's order (first group, then second)
template <bool G1, int M>
__device__ __forceinline__ void gsum_contact(const GList<M>& g, const float* cslot, float eps,
                                             v3& a, q4& r, bool rot4) {
  BX_IEEE_IN_CONTACT
  if constexpr (G1) {
    // one group: the two-group form below with its second accumulator all
    // exact zeros (0 / eps = 0, x + 0 = x), so the same bits at half the work
    v3 a0 = mk(0.f, 0.f, 0.f);
    q4 r0{0.f, 0.f, 0.f, 0.f};
    float c0 = 0.f;
#pragma unroll
    for (int k = 0; k < M; k++) {
      v3 v;
      q4 q;
      float f;
      ld_slot(cslot + (g.e[k] & 0xFFFFFF) * SLOT_STRIDE, v, q, f);
      if (!rot4) q = q4{0.f, q.w, q.x, q.y};
      a0 = a0 + v;
      r0 = r0 + q;
      c0 += f;
    }
    const float d0 = eps + c0;
    a = a0 / d0;
    r = q4{r0.w / d0, r0.x / d0, r0.y / d0, r0.z / d0};
    return;
  }
  const int g0 = g.e[0] >> 24;
  v3 a0 = mk(0.f, 0.f, 0.f), a1 = mk(0.f, 0.f, 0.f);
  q4 r0{0.f, 0.f, 0.f, 0.f}, r1{0.f, 0.f, 0.f, 0.f};
  float c0 = 0.f, c1 = 0.f;
#pragma unroll
  for (int k = 0; k < M; k++) {
    const float* s = cslot + (g.e[k] & 0xFFFFFF) * SLOT_STRIDE;
    float m0 = (g.e[k] >> 24) == g0 ? 1.f : 0.f;
    float m1 = 1.f - m0;
    v3 v;
    q4 q;
    float f;
    ld_slot(s, v, q, f);
    if (!rot4) q = q4{0.f, q.w, q.x, q.y};
    a0 = a0 + v * m0;
    a1 = a1 + v * m1;
    r0 = r0 + q * m0;
    r1 = r1 + q * m1;
    c0 += f * m0;
    c1 += f * m1;
  }
  float d0 = eps + c0, d1 = eps + c1;
  a = a0 / d0 + a1 / d1;
  r = q4{r0.w / d0 + r1.w / d1, r0.x / d0 + r1.x / d1, r0.y / d0 + r1.y / d1,
         r0.z / d0 + r1.z / d1};
}

// Euler.velocity_projection (integrators.py:122-146) on one body
__device__ __forceinline__ void vproj(QP& q, v3 ppos, q4 prot, const BodyC& B, float h,
                                      bool bare = false, bool fast = false) {
  BX_IEEE_IN_BODY
  q4 nr = bare ? qnormalize_bare(q.rot) : qnormalize(q.rot, fast);
  // (the quotients by h Newton-corrected, as qnormalize's; the Ant env
  // kernel's bare path keeps the fast ones: its 1 / h = 200 is exact)
  // (every non-bare path, both translation units: Newton-corrected
  // quotients, pbd_math.h qnormalize)
  const bool nd = !bare && !fast;  // (fast: the MULTI kernel, pbd_math.h qnormalize)
  q.vel = mul(nd ? ndiv3(q.pos - ppos, h) : (q.pos - ppos) / h, B.pm);
  q4 dq = quat_mul(nr, quat_inv(prot));
  v3 a = nd ? ndiv3(2.f * mk(dq.x, dq.y, dq.z), h) : 2.f * mk(dq.x, dq.y, dq.z) / h;
  float scl = dq.w >= 0.f ? 1.f : -1.f;
  q.ang = mul(mul(scl * B.rm, a), B.rm);
  q.rot = nr;
}

#ifdef BX_STAMPS
// per-workgroup accumulators (no atomics: contended atomics inside the timed
// windows distort them); summed on the host by debug_stamps
__device__ unsigned long long bx_stamp_wave[4096][16];
#define BX_STAMP(k)                                                                \
  do {                                                                             \
    __builtin_amdgcn_sched_barrier(0);                                             \
    unsigned long long _t;                                                         \
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(_t)::"memory");     \
    __builtin_amdgcn_sched_barrier(0);                                             \
    st_acc[k] += _t - st_last;                                                     \
    st_last = _t;                                                                  \
  } while (0)
// kernel-level stamps (env_step_kernel): slots 10..14; with BX_PSTAMPS the
// prologue's parts too (slots 5..9, BX_KSTAMP(5..9); the pbd phases' slots
// 0..9 are then not written)
#define BX_KSTAMP_DECL                                                             \
  unsigned long long kst_last, kst_acc[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0};       \
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(kst_last)::"memory");
#define BX_KSTAMP(k)                                                               \
  do {                                                                             \
    __builtin_amdgcn_sched_barrier(0);                                             \
    unsigned long long _t;                                                         \
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(_t)::"memory");     \
    __builtin_amdgcn_sched_barrier(0);                                             \
    kst_acc[(k) - 5] += _t - kst_last;                                             \
    kst_last = _t;                                                                 \
    if ((k) == 14 && threadIdx.x == 0)                                             \
      for (int _i = BX_KSLOT0; _i < 10; _i++) bx_stamp_wave[blockIdx.x & 4095][5 + _i] += kst_acc[_i]; \
  } while (0)
#if defined(BX_PSTAMPS)
#define BX_KSLOT0 0
#define BX_PSTAMP(k) BX_KSTAMP(k)
#else
#define BX_KSLOT0 5
#define BX_PSTAMP(k) do {} while (0)
#endif
#elif defined(BX_PHASE_MARKS)
// static per-phase instruction mix (diagnostic, tools/phase_mix.py): the
// stamp points as assembly comments the scheduler does not move code across
#define BX_STAMP(k)                                                                \
  do {                                                                             \
    __builtin_amdgcn_sched_barrier(0);                                             \
    asm volatile(";BXPHASE " #k ::: "memory");                                     \
    __builtin_amdgcn_sched_barrier(0);                                             \
  } while (0)
#define BX_KSTAMP_DECL
#define BX_KSTAMP(k) BX_STAMP(k)
#define BX_PSTAMP(k) do {} while (0)
#else
#define BX_STAMP(k) do {} while (0)
#define BX_KSTAMP_DECL
#define BX_KSTAMP(k) do {} while (0)
#define BX_PSTAMP(k) do {} while (0)
#endif

// FOLD (the Ant / Humanoid / HalfCheetah env kernels; the host checks that every joint j
// has torque actuator j): each joint's damping torque is added into its
// actuator's slot, so the body phase gathers one list instead of two. The
// actuator slots then no longer hold the actuators alone, which only
// System.step's Info reads.
// NOINFO (the env kernels, which write no Info): a capsule-capsule row whose
// capsule centres lie farther apart than its reach cannot penetrate, and is
// left out of the capsule-capsule pass before the segment-segment test
// FULL: every lane has a joint side, an actuator and a body copy, the `has`
// tests compile-time true. (Tried for the Ant kernel, 16 lanes = 8 joints x 2
// sides: 190 fewer SALU per step, no faster — a wave's SALU issue hides
// behind its VALU — and the merged blocks contract differently; unused.)
template <int L, int F, int M, bool FOLD = false, bool NOINFO = false, bool FULL = false>
__device__ void pbd_step_single(const Cst& c, const BlobHdr& H, const Env& E, int lane, bool valid,
                                const float* act, int aw, const Hoist<M, cl_width<F, M>()>& X,
                                v3& icv, v3& ica, v3& iaa) {
  static_assert(!FULL || ((F & F_JH) != 0 && L == 16), "FULL: the 16-lane joint halves");
  const bool hasB = FULL || X.hasB, hasJ = FULL || X.hasJ, hasA = FULL || X.hasA;
#ifdef BX_STAMPS
  unsigned long long st_acc[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
  unsigned long long st_last;
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(st_last)::"memory");
#endif
  const float h = H.h;
  const v3 g = mk(H.gx, H.gy, H.gz);
  constexpr bool JH = (F & F_JH) != 0;
  // revolute-only kernels take the atan2-free hinge (hinge_turn) on the
  // hoisted limit row. Kernels with spherical joints have no registers for
  // three rows (hoisting them: 256 VGPRs + 548 B of scratch, Humanoid 74.5 ->
  // 70.5 M env-steps/s): they read the rows from the lane image where they
  // test them (ld_lim), and take the pseudo-angle limit tests for the
  // spherical rows and torque cuts too (Humanoid 75.0 -> 78.9 M)
  // (passed by value: a pointer into X kept the hoisted struct in scratch,
  // 672-720 B per lane in every revolute kernel without joint halves)
  constexpr bool JLH = (F & F_SPH) == 0;
  const uint4* LIP = (F & F_SPH) != 0 ? E.jlim + lane : nullptr;  // staged by stage_lim
  // JH: this lane's joint / actuator and its side (lanes j and j + 8 of the
  // env's 16)
  const int jx = lane & 7;
  const bool child = (lane & 8) != 0;
  static_assert(!JH || (L == 16 && (F & F_SPH) == 0), "joint halves: revolute joints at 16 lanes");
  // JB (the Ant / HalfCheetah env kernels: joint halves, damping folded):
  // the lane's body is its side's, every side lane updating its own copy
  // with the same instructions and inputs (the side body's constants and
  // gather lists), so the copies stay bit-identical and the actuator and
  // joint phases read the state from registers, not from the LDS record the
  // previous phase wrote; the records are written where the contact passes,
  // the observation and the outputs read them (by every copy: same-address
  // writes of equal values; one writing copy per body measured slower).
  // Bodies on no joint side are frozen (checked on the host) and keep their
  // loaded record
  // (no body copies with 16-entry contact lists: Pusher folds only)
  constexpr bool JB = FOLD && JH && (F & F_C16) == 0;
  const int bi = JB ? X.S.body : lane;  // the lane's body
  float* myqp = E.qp + bi * QP_STRIDE;
  QP q;
  if (hasB) q = ldqp(myqp);
  if constexpr (JB) {
    // the records of bodies on no joint side (frozen, on the plane side of
    // one-way rows only: checked on the host) as their own lanes would leave
    // them: the previous-substep slot at their (unchanging) pose, zero contact
    // sums; the side bodies' copies overwrite their own records below
    if (lane < H.N) {
      const float* r = E.qp + lane * QP_STRIDE;
      const QP o = ldqp(r);
      st_slot(E.prev + lane * PREV_STRIDE, o.pos, o.rot, 0.f);
      st_rb(E.rb + lane * RB_STRIDE, o.pos, o.vel, o.ang);
      float* acc = E.acc + lane * ACC_STRIDE;
      st3(acc + ACC_ICV, mk(0.f, 0.f, 0.f));
      st3(acc + ACC_ICA, mk(0.f, 0.f, 0.f));
      st3(acc + ACC_IAA, mk(0.f, 0.f, 0.f));
    }
  }
  icv = mk(0.f, 0.f, 0.f);
  ica = mk(0.f, 0.f, 0.f);
  iaa = mk(0.f, 0.f, 0.f);
  // action values of the lane's actuator (constant over the step)
  float al[3] = {0.f, 0.f, 0.f};
  if (hasA && valid) {
#pragma unroll
    for (int l = 0; l < 3; l++) {
      int ai = X.A.idx[l];
      al[l] = act[take_idx(ai, aw)] * (ai >= 0 ? 1.f : 0.f);
    }
  }
  // dp_f of the lane's body: constant over the step (depends on the action only)
  v3 fv = mk(0.f, 0.f, 0.f), fa = mk(0.f, 0.f, 0.f);
  if constexpr ((F & F_FORCE) != 0) {
    if (hasB) body_forces(c, H, lane, act, aw, valid, fv, fa);
  }
  for (int it = 0; it < H.substeps / 2; it++) {
    v3 ppos = q.pos;
    q4 prot = q.rot;
    v3 dpa_last = mk(0.f, 0.f, 0.f);
#if defined(BX_SUB_UNROLL)
#pragma unroll
#else
#pragma unroll 1
#endif
    for (int sub = 0; sub < 2; sub++) {
      ppos = q.pos;
      prot = q.rot;
      if (sub == 1 && hasB) st_slot(E.prev + bi * PREV_STRIDE, ppos, prot, 0.f);
      // actuators + damping (actuator a drives joint a when H.act_same)
      if constexpr (JH) {
        // one side of joint / actuator jx per lane (act_same, checked on the host)
        const int jb = X.S.body;
        if constexpr (JB) {
          // the partner lane holds the joint's other body
          const JointC& Jc = X.J;
          const v3 oa = xh3(q.ang);
          const v3 tqd = -1.f * Jc.damping * (sel3(child, oa, q.ang) - sel3(child, q.ang, oa));
          if (hasA) act_torque_half<F>(X.J, X.JL, X.S, X.A, E, al, jx, child, q.rot, &tqd);
        } else if constexpr (FOLD) {
          const JointC& Jc = X.J;
          const v3 tqd = -1.f * Jc.damping * (ld_ang(E.qp + Jc.bp * QP_STRIDE) - ld_ang(E.qp + Jc.bc * QP_STRIDE));
          if (hasA) act_torque_half<F>(X.J, X.JL, X.S, X.A, E, al, jx, child, ld_rot(E.qp + jb * QP_STRIDE), &tqd);
        } else {
        if (hasA) act_torque_half<F>(X.J, X.JL, X.S, X.A, E, al, jx, child, ld_rot(E.qp + jb * QP_STRIDE));
        }
        if (!FOLD && hasJ) {
          const JointC& Jc = X.J;
          v3 tq = -1.f * Jc.damping * (ld_ang(E.qp + Jc.bp * QP_STRIDE) - ld_ang(E.qp + Jc.bc * QP_STRIDE));
          // parent: Ip tq, child: -Ic tq
          st_v3a(E.jslot + (child ? E.nJ + jx : jx) * SLOT_STRIDE, X.S.sg * mul(X.S.I, tq));
        }
      } else {
      if (hasA) {
        const ActC& A = X.A;
        if (FOLD) {
          const JointC& Jc = X.J;
          const v3 tqd = -1.f * Jc.damping * (ld_ang(E.qp + Jc.bp * QP_STRIDE) - ld_ang(E.qp + Jc.bc * QP_STRIDE));
          act_torque<F, L>(X.J, A, E, al, lane, JLH, X.JL, LIP, &tqd);
        } else if (H.act_same) {
          act_torque<F, L>(X.J, A, E, al, lane, JLH, X.JL, LIP);
        } else {
          JointC Jc = load_joint(c, H, A.joint);
          act_torque<F>(Jc, A, E, al, lane);
        }
      }
      if (!FOLD && hasJ) {
        const JointC& Jc = X.J;
        v3 tq = -1.f * Jc.damping * (ld_ang(E.qp + Jc.bp * QP_STRIDE) - ld_ang(E.qp + Jc.bc * QP_STRIDE));
        st_v3a(E.jslot + lane * SLOT_STRIDE, mul(Jc.Ip, tq));
        st_v3a(E.jslot + (E.nJ + lane) * SLOT_STRIDE, -1.f * mul(Jc.Ic, tq));
      }
      }
      phase_sync();
      BX_STAMP(0);
      if (hasB) {
        v3 dpa = gsum3(X.al, E.aslot, ASLOT_STRIDE);
        v3 dpj = FOLD ? mk(0.f, 0.f, 0.f) : gsum3(X.jl, E.jslot, SLOT_STRIDE);
        v3 vel = H.vexp * q.vel;
        vel = vel + (fv + g) * h;
        q.vel = mul(vel, X.B.pm);
        v3 an = H.aexp * q.ang;
        an = an + ((dpa + fa) + dpj) * h;
        q.ang = mul(an, X.B.rm);
        q.pos = q.pos + mul(q.vel * h, X.B.pm);
        v3 am = mul(q.ang, X.B.rm);
        q4 hq = (q4{0.f, am.x, am.y, am.z} * 0.5f) * h;
        q4 r = q.rot + quat_mul(hq, q.rot);
        q.rot = JB ? qnormalize_bare(r) : qnormalize(r);  // Ant env kernel: bare sqrt
        if (!JB) stqp(myqp, q);  // JB: the joint phase takes the lane's copy
        dpa_last = dpa;
      }
      phase_sync();
      BX_STAMP(1);
      if constexpr (JH) {
        if (hasJ) {
          const JointC& Jc = X.J;
          const QP o = JB ? q : ldqp(E.qp + X.S.body * QP_STRIDE);
          v3 dpo;
          q4 dro;
          joint_apply_half(Jc, X.JL, X.S, child, o, dpo, dro);
          st_slot(E.jslot + (child ? E.nJ + jx : jx) * SLOT_STRIDE, dpo, dro, 0.f);
        }
      } else if (hasJ) {
        const JointC& Jc = X.J;
        QP p = ldqp(E.qp + Jc.bp * QP_STRIDE), cq = ldqp(E.qp + Jc.bc * QP_STRIDE);
        v3 dpp, dcp;
        q4 dpr, dcr;
        joint_apply<F, L>(Jc, p, cq, dpp, dpr, dcp, dcr, JLH, X.JL, LIP);
        st_slot(E.jslot + lane * SLOT_STRIDE, dpp, dpr, 0.f);
        st_slot(E.jslot + (E.nJ + lane) * SLOT_STRIDE, dcp, dcr, 0.f);
      }
      phase_sync();
      BX_STAMP(2);
      if (hasB) {
        v3 dp = mk(0.f, 0.f, 0.f);
        q4 dr{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int k = 0; k < M; k++) {
          v3 v;
          q4 r;
          float f;
          ld_slot(E.jslot + X.jl.e[k] * SLOT_STRIDE, v, r, f);
          dp = dp + v;
          dr = dr + r;
        }
        q.pos = q.pos + mul(dp, X.B.pm);
        q.rot = q4{q.rot.w + dr.w * X.B.qm.w, q.rot.x + dr.x * X.B.qm.x, q.rot.y + dr.y * X.B.qm.y,
                   q.rot.z + dr.z * X.B.qm.z};
        if (sub == 0) vproj(q, ppos, prot, X.B, h, JB);
        // JB: the record is read next by the contact passes (after sub 1)
        if (!JB || sub == 1) stqp(myqp, q);
      }
      phase_sync();
      BX_STAMP(3);
    }
    // ---- collisions (system.py:288-313): the lane's row (F_R2: rows lane
    // and lane + 16), its contact kept in registers until the velocity pass
    constexpr bool R2 = (F & F_R2) != 0;
    v3 cpos = mk(0.f, 0.f, 0.f), cn = mk(0.f, 0.f, 0.f);
    float pen = 0.f, dl = 0.f;
    v3 cpos2 = mk(0.f, 0.f, 0.f), cn2 = mk(0.f, 0.f, 0.f);
    float pen2 = 0.f, dl2 = 0.f;
    // F_R2G: slot 1 holds only one-way capsule-plane rows, slot 2 only
    // two-way capsule-capsule rows
    constexpr bool RG = (F & F_R2G) != 0;
    constexpr int F1 = RG ? (F & ~(F_CC | F_TW)) : F;
    constexpr int F2 = RG ? (F | F_CCO) : F;
    // a row that does not penetrate (pen <= 0) has c >= 0 in the position
    // pass (cm = 0) and sm = 0 in the velocity pass: its impulses are exact
    // zeros. The passes with capsule-capsule code (pairs that rarely touch)
    // skip that math for such rows, and a wave in which no row of the pass
    // penetrates skips it whole (the branch's exec mask is empty); the
    // plane passes (some foot of the wave's envs is down at almost every
    // substep) keep the straight-line code
    const v3 z3 = mk(0.f, 0.f, 0.f);
    const q4 z4{0.f, 0.f, 0.f, 0.f};
    auto pos_pass = [&](auto fc, const RowC& R, int r, v3& cpos, v3& cn, float& pen, float& dl) {
      constexpr int FS = decltype(fc)::value;
      QP a = ldqp(E.qp + R.a * QP_STRIDE), b = ldqp(E.qp + R.b * QP_STRIDE);
      v3 cvel;
      bool far = false;
      if constexpr (NOINFO && (FS & F_CCO) != 0) {
        // the closest points lie within half a segment of each centre, so
        // dist >= |centre_a - centre_b| - |end_a| - |end_b|; reach rounded up
        const v3 d = (a.pos + rotate(R.a_pos, a.rot)) - (b.pos + rotate(R.b_pos, b.rot));
        const float reach =
            (norm(R.a_end) + norm(R.b_end) + R.a_rad + R.b_rad) * 1.00001f + 1e-4f;
        const float dd = dot(d, d);
        far = dd > reach * reach && !is_nan(dd);
      }
      if (far) {
        cpos = z3;
        cn = z3;
        pen = -1.f;
      } else {
        contact_gen<FS>(R, a, b, cpos, cvel, cn, pen);
      }
      if constexpr (HALF<FS>()) {
        // contact halves: this lane's side only (a on lanes 0-7, b on 8-15)
        const bool sb = (lane & 8) != 0;
        v3 pop, op = z3;
        q4 por, orr = z4;
        float unused;
        ld_slot(E.prev + (sb ? R.b : R.a) * PREV_STRIDE, pop, por, unused);
        if (is_nan(pen)) {
          const float pz = nan_of(pen);
          op = mk(pz, pz, pz);
          orr = q4{pz, pz, pz, pz};
          dl = pz;
        } else if (pen > 0.f) {
          dl = position_contact_half<FS>(R, sb ? b : a, pop, por, cpos, cn, pen, sb, op, orr);
        } else {
          dl = 0.f;
        }
        if (!sb) {
          float* rd = E.rowd + r * ROWD_STRIDE;
          st4a(rd, f32x4{cpos.x, cpos.y, cpos.z, cn.x});
          st4a(rd + 4, f32x4{cn.y, cn.z, pen, dl});
        }
        st_slot(E.cslot + (sb ? E.nR + r : r) * SLOT_STRIDE, op, orr, nonzero3(op));
        return;
      }
      v3 pap, pbp;
      q4 par, pbr;
      float unused;
      ld_slot(E.prev + R.a * PREV_STRIDE, pap, par, unused);
      ld_slot(E.prev + R.b * PREV_STRIDE, pbp, pbr, unused);
      v3 oap = z3, obp = z3;
      q4 oar = z4, obr = z4;
      if ((FS & F_CC) != 0 && is_nan(pen)) {
        // a NaN contact's impulses are NaN on both sides (the reference's
        // masked products, colliders.py:332-333: NaN * 0)
        const float pz = nan_of(pen);
        oap = obp = mk(pz, pz, pz);
        oar = obr = q4{pz, pz, pz, pz};
        dl = pz;
      } else if (!((FS & F_CC) != 0) || pen > 0.f) {
        dl = position_contact<FS>(R, a, b, pap, par, pbp, pbr, cpos, cn, pen, oap, oar, obp, obr);
      } else {
        dl = 0.f;
      }
      float* rd = E.rowd + r * ROWD_STRIDE;
      st4a(rd, f32x4{cpos.x, cpos.y, cpos.z, cn.x});
      st4a(rd + 4, f32x4{cn.y, cn.z, pen, dl});
      st_slot(E.cslot + r * SLOT_STRIDE, oap, oar,
              nonzero3(oap));
      st_slot(E.cslot + (E.nR + r) * SLOT_STRIDE, obp, obr,
              nonzero3(obp));
    };
    if (X.hasR) pos_pass(std::integral_constant<int, F1>{}, X.R, X.r1, cpos, cn, pen, dl);
    if constexpr (R2) {
      if (X.hasR2) pos_pass(std::integral_constant<int, F2>{}, X.R2, X.r2, cpos2, cn2, pen2, dl2);
    }
    phase_sync();
    BX_STAMP(4);
    if (hasB) {
      v3 dp;
      q4 dr;
      gsum_contact<(F & F_G1) != 0>(X.cl, E.cslot, 1e-6f, dp, dr, true);
      q.pos = q.pos + mul(dp, X.B.pm);
      q.rot = q4{q.rot.w + dr.w * X.B.qm.w, q.rot.x + dr.x * X.B.qm.x, q.rot.y + dr.y * X.B.qm.y,
                 q.rot.z + dr.z * X.B.qm.z};
      st_rb(E.rb + bi * RB_STRIDE, q.pos, q.vel, q.ang);
      vproj(q, ppos, prot, X.B, h, JB);
      stqp(myqp, q);
    }
    phase_sync();
    BX_STAMP(5);
    auto vel_pass = [&](auto fc, const RowC& R, int r, v3 cpos, v3 cn, float pen, float dl) {
      constexpr int FS = decltype(fc)::value;
      if constexpr (HALF<FS>()) {
        const bool sb = (lane & 8) != 0;
        const QP o = ldqp(E.qp + (sb ? R.b : R.a) * QP_STRIDE);
        v3 rop, rov, roa, ov = z3, oa = z3;
        ld_rb(E.rb + (sb ? R.b : R.a) * RB_STRIDE, rop, rov, roa);
        if (is_nan(pen)) {
          const float pz = nan_of(pen);
          ov = oa = mk(pz, pz, pz);
        } else if (pen > 0.f) {
          velocity_contact_half<FS>(R, h, o, rop, rov, roa, cpos, cn, pen, dl, sb, ov, oa);
        }
        st_slot(E.cslot + (sb ? E.nR + r : r) * SLOT_STRIDE, ov, q4{oa.x, oa.y, oa.z, 0.f}, nonzero3(ov));
        return;
      }
      QP a = ldqp(E.qp + R.a * QP_STRIDE), b = ldqp(E.qp + R.b * QP_STRIDE);
      v3 rap, rav, raa, rbp, rbv, rba;
      ld_rb(E.rb + R.a * RB_STRIDE, rap, rav, raa);
      ld_rb(E.rb + R.b * RB_STRIDE, rbp, rbv, rba);
      v3 oav = z3, oaa = z3, obv = z3, oba = z3;
      if ((FS & F_CC) != 0 && is_nan(pen)) {
        const float pz = nan_of(pen);
        oav = oaa = obv = oba = mk(pz, pz, pz);
      } else if (!((FS & F_CC) != 0) || pen > 0.f) {
        velocity_contact<FS>(R, h, a, b, rap, rav, raa, rbp, rbv, rba, cpos, cn, pen, dl, oav, oaa,
                             obv, oba);
      }
      st_slot(E.cslot + r * SLOT_STRIDE, oav, q4{oaa.x, oaa.y, oaa.z, 0.f},
              nonzero3(oav));
      st_slot(E.cslot + (E.nR + r) * SLOT_STRIDE, obv, q4{oba.x, oba.y, oba.z, 0.f},
              nonzero3(obv));
    };
    if (X.hasR) vel_pass(std::integral_constant<int, F1>{}, X.R, X.r1, cpos, cn, pen, dl);
    if constexpr (R2) {
      if (X.hasR2) vel_pass(std::integral_constant<int, F2>{}, X.R2, X.r2, cpos2, cn2, pen2, dl2);
    }
    phase_sync();
    BX_STAMP(6);
    if (hasB) {
      v3 dv;
      q4 da;
      gsum_contact<(F & F_G1) != 0>(X.cl, E.cslot, 1e-6f, dv, da, false);
      v3 dav = mk(da.x, da.y, da.z);
      q.vel = mul(q.vel + dv, X.B.pm);
      q.ang = mul(q.ang + dav, X.B.rm);
      stqp(myqp, q);
      icv = icv + dv;
      ica = ica + dav;
      iaa = iaa + dpa_last;
    }
    phase_sync();
    BX_STAMP(7);
  }
  if (hasB) {
    // a NaN body's contact Info is NaN when it has contact rows: its rows'
    // masked impulses were NaN (colliders.py:332-333, 440-442: NaN * 0; the
    // straight-line plane passes above fold the masks to selects, so the
    // slots carried zeros). A body's state is NaN at the end of the step
    // exactly when a contact pass of the step saw it NaN (a one-way row's
    // contact is its body's; the two-way passes carry NaN rows explicitly)
    if ((X.cl.e[0] & 0xFFFFFF) != 2 * H.R) {
      const float pz = nan_of(((q.pos.x + q.pos.y) + (q.pos.z + q.rot.w)) +
                              ((q.rot.x + q.rot.y) + (q.rot.z + q.vel.x)) +
                              ((q.vel.y + q.vel.z) + (q.ang.x + q.ang.y)) + q.ang.z);
      icv = icv + mk(pz, pz, pz);
      ica = ica + mk(pz, pz, pz);
    }
    float* acc = E.acc + bi * ACC_STRIDE;
    st3(acc + ACC_ICV, icv);
    st3(acc + ACC_ICA, ica);
    st3(acc + ACC_IAA, iaa);
  }
  phase_sync();
  BX_STAMP(9);
#ifdef BX_STAMPS
  if (threadIdx.x == 0) {
#if !defined(BX_PSTAMPS)
#pragma unroll
    for (int k = 0; k < 10; k++) bx_stamp_wave[blockIdx.x & 4095][k] += st_acc[k];
#endif
    bx_stamp_wave[blockIdx.x & 4095][15] += 1ull;
  }
#endif
}

// ---------------------------------------------------------------------------
// MULTI mode: large pbd scenes (Ant Mountain: 37 bodies, 32 joints, 702
// contact rows). One env per 256-thread workgroup (4 waves, workgroup
// barriers between phases). Lane l owns body l, joint l and actuator l with
// their constants hoisted into registers (as SINGLE mode), contact rows l,
// l + L, ... (<= MR, constants hoisted, the row's contact kept in registers
// between the position and velocity passes) and gather task l. The
// reference's per-body segment_sums over up to ~40 contact rows become two
// short fixed-order phases: each task sums <= TASK_W slots of one body and
// collider group into a partial, then each body adds its <= BTASK_W partials
// group by group, each group divided by (eps + count) (colliders.py:198-240).
// ---------------------------------------------------------------------------
struct HoistM {
  bool hasB, hasJ, hasA;
  BodyC B;
  JointC J;  // joint halves (MJH): the lane's joint side's joint
  ActC A;
  JSide S;   // MJH: the lane's side, its joint's first limit row
  JLim JL;
  // the body's joint / actuator slot lists (padding: the zero slots), two
  // 16-bit entries per word (registers are the MULTI kernel's limit: 256 at
  // two waves per SIMD)
  uint32_t jl[MAXG / 2], al[MAXG / 2];
  // the lane's two tasks (lane, lane + L): TASK_W entries each (row | side
  // << 15; padding: row R), two 16-bit entries per word
  uint32_t te[2][TASK_W / 2];
  // the lane's body: task | group << 10 (padding: the zero task), 16-bit pairs
  uint32_t bt[BTASK_W / 2];
};
__device__ __forceinline__ int ent16(const uint32_t* p, int k) {
  return (int)((p[k >> 1] >> ((k & 1) * 16)) & 0xFFFFu);
}
template <int M>
__device__ __forceinline__ v3 gsum3p(const uint32_t* g, const float* base, int stride) {
  v3 s = mk(0.f, 0.f, 0.f);
#pragma unroll
  for (int k = 0; k < M; k++) s = s + ld_v3a(base + ent16(g, k) * stride);
  return s;
}
// MJH: the lane's joint side from the MULTI joint-halves image (MJ_*, 20
// independent 16-byte loads), parsed as the SINGLE lane image's records
__device__ __forceinline__ void load_mjh(const Cst& c, const BlobHdr& H, int lane, HoistM& X) {
  const int jx = ((lane >> 4) << 3) + (lane & 7);
  X.hasJ = jx < H.J;
  X.hasA = jx < H.K;
  const uint4* im = reinterpret_cast<const uint4*>(c.w + H.o_mjh) + lane;
  uint32_t w[MJ_W];
#pragma unroll
  for (int g = 0; g < MJ_W / 4; g++) {
    const uint4 v = im[g * MJ_LANES];
    w[4 * g] = v.x; w[4 * g + 1] = v.y; w[4 * g + 2] = v.z; w[4 * g + 3] = v.w;
  }
  auto f = [&](int i) { return __uint_as_float(w[i]); };
  auto f3 = [&](int i) { return mk(f(i), f(i + 1), f(i + 2)); };
  auto n = [&](int i) { return (int)w[i]; };
  JointC& J = X.J;
  constexpr int OJ = MJ_JOINT;
  J.type = n(OJ + LJ_TYPE);
  J.bp = n(OJ + LJ_BP);
  J.bc = n(OJ + LJ_BC);
  J.free = n(OJ + LJ_FREE);
  J.angle_off = n(OJ + LJ_AOFF);
  J.n_angles = n(OJ + LJ_NANG);
  J.dof = n(OJ + LJ_DOF);
  J.damping = f(OJ + LJ_DAMP);
  J.sp = f(OJ + LJ_SP);
  J.sa = f(OJ + LJ_SA);
  J.off_p = f3(OJ + LJ_OFFP);
  J.off_c = f3(OJ + LJ_OFFC);
#pragma unroll
  for (int k = 0; k < 3; k++) {
    J.axp[k] = f3(OJ + LJ_AXP + 3 * k);
    J.axc[k] = f3(OJ + LJ_AXC + 3 * k);
  }
#pragma unroll
  for (int k = 0; k < 6; k++) J.lim[k] = f(OJ + LJ_LIM + k);
  J.mp = f(OJ + LJ_MP);
  J.mc = f(OJ + LJ_MC);
  J.Ip = f3(OJ + LJ_IP);
  J.Ic = f3(OJ + LJ_IC);
  X.A.type = n(MJ_ACT + LA_TYPE);
  X.A.joint = n(MJ_ACT + LA_JOINT);
#pragma unroll
  for (int k = 0; k < 3; k++) X.A.idx[k] = n(MJ_ACT + LA_IDX + k);
  X.A.strength = f(MJ_ACT + LA_STR);
  constexpr int OL = MJ_JLIM;
  X.JL = JLim{f(OL + LL_PLO), f(OL + LL_PHI), f(OL + LL_CLO), f(OL + LL_SLO), f(OL + LL_CHI),
              f(OL + LL_SHI)};
  X.S.off = f3(MJ_SIDE + LS_OFF);
  X.S.ax0 = f3(MJ_SIDE + LS_AX0);
  X.S.ax2 = f3(MJ_SIDE + LS_AX2);
  X.S.I = f3(MJ_SIDE + LS_I);
  X.S.m = f(MJ_SIDE + LS_M);
  X.S.sg = f(MJ_SIDE + LS_SG);
  X.S.body = n(MJ_SIDE + LS_BODY);
}

template <int L, bool MJH = false>
__device__ __forceinline__ void load_hoist_multi(const Cst& c, const BlobHdr& H, int lane,
                                                 HoistM& X) {
  X.hasB = lane < H.N;
  X.hasJ = lane < H.J;
  X.hasA = lane < H.K;
  const int b = X.hasB ? lane : 0;
  X.B = load_body(c, H, b);
  {
    const GList<MAXG> jl = load_glist<MAXG>(c, H.o_jl_off, H.o_jl, b, X.hasB, 2 * H.J);
    const GList<MAXG> al = load_glist<MAXG>(c, H.o_al_off, H.o_al, b, X.hasB, 2 * H.K);
#pragma unroll
    for (int k = 0; k < MAXG / 2; k++) {
      X.jl[k] = (uint32_t)jl.e[2 * k] | ((uint32_t)jl.e[2 * k + 1] << 16);
      X.al[k] = (uint32_t)al.e[2 * k] | ((uint32_t)al.e[2 * k + 1] << 16);
    }
  }
#pragma unroll
  for (int q = 0; q < 2; q++) {
    const int t = lane + q * L;
    const bool hasT = t < H.T;
#pragma unroll
    for (int k = 0; k < TASK_W / 2; k++) {
      const uint32_t lo = hasT ? (uint32_t)c.i(H.o_task + t * TASK_W + 2 * k) : (uint32_t)H.R;
      const uint32_t hi = hasT ? (uint32_t)c.i(H.o_task + t * TASK_W + 2 * k + 1) : (uint32_t)H.R;
      X.te[q][k] = lo | (hi << 16);
    }
  }
#pragma unroll
  for (int k = 0; k < BTASK_W / 2; k++) {
    uint32_t w[2];
#pragma unroll
    for (int i = 0; i < 2; i++) {
      const uint32_t v = X.hasB ? (uint32_t)c.i(H.o_btask + b * BTASK_W + 2 * k + i) : (uint32_t)H.T;
      w[i] = (v & 0x3FFu) | ((v >> 24) << 10);
    }
    X.bt[k] = w[0] | (w[1] << 16);
  }
  if constexpr (MJH) {
    load_mjh(c, H, lane, X);
  } else {
    if (H.J > 0) X.J = load_joint(c, H, X.hasJ ? lane : 0);
    if (H.K > 0) X.A = load_act(c, H, X.hasA ? lane : 0);
  }
}

// phase 1: a task's partial, its entries summed in list order; an entry
// counts when its linear part is nonzero (the reference's any(dq_pos) /
// any(dp_vel) per row, colliders.py:187-195,231-239). An entry is a row and
// side: its slot in chunk ch is the row's compact index less the chunk's
// first, on the side's half, when the row is listed in this chunk, else the
// zero slot (the rows without an update). Chunks after the first add to
// the partial (one chunk: the sum of every entry's slot in list order, as
// when every row had a slot)
__device__ __forceinline__ void task_sum(const uint32_t* te, const uint16_t* sidx, const float* ms,
                                         float* out, int ch) {
  v3 a = mk(0.f, 0.f, 0.f), l = mk(0.f, 0.f, 0.f);
  float n = 0.f;
  if (ch > 0) {
    const f32x4 t0 = ld4a(out), t1 = ld4a(out + 4);
    a = mk(t0[0], t0[1], t0[2]);
    l = mk(t0[3], t1[0], t1[1]);
    n = t1[2];
  }
  int slot[TASK_W];
#pragma unroll
  for (int k = 0; k < TASK_W; k++) {
    const uint32_t e = (te[k >> 1] >> ((k & 1) * 16)) & 0xFFFFu;
    const uint32_t rel = (uint32_t)sidx[e & 0x7FFFu] - (uint32_t)(ch * MCAP);
    slot[k] = rel < (uint32_t)MCAP ? (int)rel + (int)(e >> 15) * MCAP : 2 * MCAP;
  }
#pragma unroll
  for (int k = 0; k < TASK_W; k++) {
    v3 v, w;
    ld_mslot(ms + slot[k] * MSLOT_STRIDE, v, w);
    a = a + v;
    l = l + w;
    n += nonzero3(v);
  }
  st4a(out, f32x4{a.x, a.y, a.z, l.x});
  st4a(out + 4, f32x4{l.y, l.z, n, 0.f});
}

// phase 2: sum over the body's groups of (group's partials) / (eps + count):
// the linear part a and the angular part l
__device__ __forceinline__ void body_combine(const uint32_t* bt, const float* ts, float eps, v3& a,
                                             v3& l) {
  a = mk(0.f, 0.f, 0.f);
  l = mk(0.f, 0.f, 0.f);
  v3 ga = mk(0.f, 0.f, 0.f), gl = mk(0.f, 0.f, 0.f);
  float gn = 0.f;
  int g = ent16(bt, 0) >> 10;
#pragma unroll
  for (int k = 0; k < BTASK_W; k++) {
    const int e = ent16(bt, k);
    const float* t = ts + (e & 0x3FF) * TSLOT_STRIDE;
    const f32x4 t0 = ld4a(t), t1 = ld4a(t + 4);
    const int gk = e >> 10;
    if (gk != g) {
      const float d = eps + gn;
      a = a + ga / d;
      l = l + gl / d;
      ga = mk(0.f, 0.f, 0.f);
      gl = mk(0.f, 0.f, 0.f);
      gn = 0.f;
      g = gk;
    }
    ga = ga + mk(t0[0], t0[1], t0[2]);
    gl = gl + mk(t0[3], t1[0], t1[1]);
    gn += t1[2];
  }
  const float d = eps + gn;
  a = a + ga / d;
  l = l + gl / d;
}

// info: the env's Info contact rows (contact_pos 3, normal 3, penetration),
// already offset to this env; null pointers are skipped
struct RowInfoOut {
  float* pos;
  float* normal;
  float* pen;
  int32_t* cell;  // the row's NearNeighbors cell (R_FLAT)
};

#ifdef BX_MSTAMPS
// MULTI-mode phase stamps of each workgroup's first wave (diagnostic build)
__device__ unsigned long long bx_mstamp_wave[4096][16];
#define BX_MSTAMP(k)                                                               \
  do {                                                                             \
    __builtin_amdgcn_sched_barrier(0);                                             \
    unsigned long long _t;                                                         \
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(_t)::"memory");     \
    __builtin_amdgcn_sched_barrier(0);                                             \
    ms_acc[k] += _t - ms_last;                                                     \
    ms_last = _t;                                                                  \
  } while (0)
#else
#define BX_MSTAMP(k) do {} while (0)
#endif

template <int L, int F>
__device__ void pbd_step_multi(const Cst& c, const BlobHdr& H, const Env& E, int lane, bool valid,
                               const float* act, int aw, const HoistM& X, RowInfoOut io,
                               float* ovf) {
#ifdef BX_MSTAMPS
  unsigned long long ms_acc[15] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
  unsigned long long ms_last;
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(ms_last)::"memory");
#endif
  const float h = H.h;
  const v3 g = mk(H.gx, H.gy, H.gz);
  // MJH (the joint halves, F_JH): the lane's joint jx and side
  constexpr bool MJH = (F & F_JH) != 0;
  constexpr int NWV = L / 64;
  const int wv = lane >> 6;
  const int mjx = ((lane >> 4) << 3) + (lane & 7);
  const bool mchild = (lane & 8) != 0;
  const bool info_rows = io.pos || io.normal || io.pen || io.cell;
  float* myqp = E.qp + lane * QP_STRIDE;
  QP q;
  if (X.hasB) q = ldqp(myqp);
  v3 icv = mk(0.f, 0.f, 0.f), ica = mk(0.f, 0.f, 0.f), iaa = mk(0.f, 0.f, 0.f);
  float al[3] = {0.f, 0.f, 0.f};
  if (X.hasA && valid) {
#pragma unroll
    for (int l = 0; l < 3; l++) {
      int ai = X.A.idx[l];
      al[l] = act[take_idx(ai, aw)] * (ai >= 0 ? 1.f : 0.f);
    }
  }
  v3 fv = mk(0.f, 0.f, 0.f), fa = mk(0.f, 0.f, 0.f);
  if constexpr ((F & F_FORCE) != 0) {
    if (X.hasB) body_forces(c, H, lane, act, aw, valid, fv, fa);
  }
  // NearNeighbors.update once per step (system.py:320-321): the selected
  // rows' ranks in E.ract, in Info order in E.alist (the culled rows have no
  // contact index, so their slots are never read)
  if (H.n_nn) {
    place_centres<L>(H, E, lane);
    esync<L>();
#ifdef BX_MSTAMPS
    nn_select<L, true, (L >= 256 ? 4 : 8)>(c, H, E, lane, ms_acc, &ms_last);
#else
    nn_select<L, true, (L >= 256 ? 4 : 8)>(c, H, E, lane);
#endif
  }
  BX_MSTAMP(9);
  // the step's work rows: row x of the culled scenes' active rows in Info
  // order (E.alist), else row x
  const int nact = H.n_nn ? H.info_rows : H.R;
#define BX_MULTI_RX(x) (H.n_nn ? E.alist[x] : (x))
  // a penetrating row's contact (compact index y): LDS below MCBUF, the env's
  // overflow slice past it
  auto cb_at = [&](int y) -> float* {
    return y < MCBUF ? E.cbuf + y * MCB_W : ovf + (int64_t)(y - MCBUF) * MOVF_W;
  };
  uint16_t* cbrow = reinterpret_cast<uint16_t*>(E.cbuf + MCBUF * MCB_W);
  auto cb_row = [&](int y) -> int {
    return y < MCBUF ? (int)cbrow[y] : __float_as_int(ovf[(int64_t)(y - MCBUF) * MOVF_W + 8]);
  };
  // the tasks' sums of chunk ch (TASK_W entries each, in list order; a partial
  // carried over from the chunk before)
  auto tasks = [&](int ch) {
#pragma unroll
    for (int k = 0; k < 2; k++) {
      const int t = lane + k * L;
      if (t < H.T) task_sum(X.te[k], E.sidx, E.cslot, E.tslot + t * TSLOT_STRIDE, ch);
    }
  };
  for (int it = 0; it < H.substeps / 2; it++) {
    v3 ppos = q.pos;
    q4 prot = q.rot;
    v3 dpa_last = mk(0.f, 0.f, 0.f);
#pragma unroll 1
    for (int sub = 0; sub < 2; sub++) {
      ppos = q.pos;
      prot = q.rot;
      if (sub == 1 && X.hasB) st_slot(E.prev + lane * PREV_STRIDE, ppos, prot, 0.f);
      // actuators (actuators.py:52-112) + joint damping (joints.py:103-128)
      if constexpr (MJH) {
        // one side of joint / actuator jx per lane: the side's damping torque
        // into its joint slot (parent: Ip tq, child: -Ic tq), its actuator
        // torque into its actuator slot
        if (X.hasJ) {
          const JointC& Jc = X.J;
          const v3 tq = -1.f * Jc.damping * (ld_ang(E.qp + Jc.bp * QP_STRIDE) - ld_ang(E.qp + Jc.bc * QP_STRIDE));
          st_v3a(E.jslot + (mchild ? E.nJ + mjx : mjx) * SLOT_STRIDE, X.S.sg * mul(X.S.I, tq));
          if (X.hasA)
            act_torque_half<F>(X.J, X.JL, X.S, X.A, E, al, mjx, mchild, ld_rot(E.qp + X.S.body * QP_STRIDE));
        }
      } else {
      if (X.hasA) {
        if (H.act_same) {
          act_torque<F>(X.J, X.A, E, al, lane);
        } else {
          JointC Jc = load_joint(c, H, X.A.joint);
          act_torque<F>(Jc, X.A, E, al, lane);
        }
      }
      if (X.hasJ) {
        const JointC& Jc = X.J;
        v3 tq = -1.f * Jc.damping * (ld_ang(E.qp + Jc.bp * QP_STRIDE) - ld_ang(E.qp + Jc.bc * QP_STRIDE));
        st_v3a(E.jslot + lane * SLOT_STRIDE, mul(Jc.Ip, tq));
        st_v3a(E.jslot + (E.nJ + lane) * SLOT_STRIDE, -1.f * mul(Jc.Ic, tq));
      }
      }
      esync<L>();
      BX_MSTAMP(0);
      // Euler.update(acc) + Euler.kinetic (integrators.py:50-93)
      if (X.hasB) {
        v3 dpa = gsum3p<MAXG>(X.al, E.aslot, ASLOT_STRIDE);
        v3 dpj = gsum3p<MAXG>(X.jl, E.jslot, SLOT_STRIDE);
        v3 vel = H.vexp * q.vel;
        vel = vel + (fv + g) * h;
        q.vel = mul(vel, X.B.pm);
        v3 an = H.aexp * q.ang;
        an = an + ((dpa + fa) + dpj) * h;
        q.ang = mul(an, X.B.rm);
        q.pos = q.pos + mul(q.vel * h, X.B.pm);
        v3 am = mul(q.ang, X.B.rm);
        q4 hq = (q4{0.f, am.x, am.y, am.z} * 0.5f) * h;
        q4 r = q.rot + quat_mul(hq, q.rot);
        q.rot = qnormalize(r, true);
        stqp(myqp, q);
        dpa_last = dpa;
      }
      esync<L>();
      BX_MSTAMP(1);
      // Joint.apply (joints.py:79-100)
      if constexpr (MJH) {
        if (X.hasJ) {
          const QP o = ldqp(E.qp + X.S.body * QP_STRIDE);
          v3 dpo;
          q4 dro;
          joint_apply_half(X.J, X.JL, X.S, mchild, o, dpo, dro);
          st_slot(E.jslot + (mchild ? E.nJ + mjx : mjx) * SLOT_STRIDE, dpo, dro, 0.f);
        }
      } else if (X.hasJ) {
        const JointC& Jc = X.J;
        QP p = ldqp(E.qp + Jc.bp * QP_STRIDE), cq = ldqp(E.qp + Jc.bc * QP_STRIDE);
        v3 dpp, dcp;
        q4 dpr, dcr;
        joint_apply<F>(Jc, p, cq, dpp, dpr, dcp, dcr);
        st_slot(E.jslot + lane * SLOT_STRIDE, dpp, dpr, 0.f);
        st_slot(E.jslot + (E.nJ + lane) * SLOT_STRIDE, dcp, dcr, 0.f);
      }
      esync<L>();
      BX_MSTAMP(2);
      // Euler.update(pos) (+ velocity_projection on the first substep)
      if (X.hasB) {
        v3 dp = mk(0.f, 0.f, 0.f);
        q4 dr{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int k = 0; k < MAXG; k++) {
          v3 v;
          q4 r;
          float f;
          ld_slot(E.jslot + ent16(X.jl, k) * SLOT_STRIDE, v, r, f);
          dp = dp + v;
          dr = dr + r;
        }
        q.pos = q.pos + mul(dp, X.B.pm);
        q.rot = q4{q.rot.w + dr.w * X.B.qm.w, q.rot.x + dr.x * X.B.qm.x, q.rot.y + dr.y * X.B.qm.y,
                   q.rot.z + dr.z * X.B.qm.z};
        if (sub == 0) vproj(q, ppos, prot, X.B, h, false, true);
        stqp(myqp, q);
      }
      esync<L>();
      BX_MSTAMP(3);
    }
    // ---- collisions (system.py:288-313)
    // Broad phase, on every pass but the step's last (whose contacts are the
    // step's Info): a capsule pair whose centres lie farther apart than its
    // reach cannot penetrate, so both its passes' updates are exact zeros;
    // the near rows are listed in (m, wave, lane) order (E.nearl) for the
    // contact pass, the far rows sit it out (no slot: no update, no count).
    // (culled scenes skip it: NearNeighbors already keeps only near cells).
    // Without contact-row Info (System.step(..., info=False): no caller
    // reads the rows) the last pass takes it too: its far rows' Info is never
    // written
    const bool last = it + 1 == H.substeps / 2;
    const int lane0 = lane;
    const bool bph = H.o_bimg != 0 && H.n_nn == 0 && (!last || !info_rows);
    int nwork = nact;
    if (bph) {
      int* cnt = E.nearc;
      // (the lane index made opaque per pass: its row addresses and masks are
      // recomputed here instead of hoisted out of the substep loop, where
      // they had no registers left and went to scratch)
      int lane = lane0;
      asm volatile("" : "+v"(lane));
      // the capsule centres in the world, once for every row naming them
      place_centres<L>(H, E, lane);
      esync<L>();
      // the lane's rows r = lane + m L (m < 8: the host keeps R <= 8 L):
      // near bits, per (m, wave) counts; unrolled, so every row's loads issue
      // together
      unsigned nmask = 0u;
      const int nm = (H.R + L - 1) / L;
#pragma unroll
      for (int m = 0; m < 8; m++) {
        if (m >= nm) break;
        const int r = lane + m * L;
        bool near = false;
        if (r < H.R) {
          const uint2 g0 = *reinterpret_cast<const uint2*>(E.bimg + r * BI_WORDS);
          near = (bi_flags(g0.x) & BIF_SKIP) == 0u;
          if (!near) {
            // squared distance against (reach + 1e-4)^2 (bx_capi.cpp); a NaN
            // distance is near (a NaN row's impulses are NaN)
            const float cd2 = centre_dist2(E, H, bi_pair(g0.x));
            near = !(cd2 > bi_reach2(g0.y)) || is_nan(cd2);
          }
        }
        nmask |= near ? (1u << m) : 0u;
        const unsigned long long bal = __ballot(near);
        if ((lane & 63) == 0) cnt[m * NWV + wv] = __popcll(bal);
      }
      esync<L>();
      int total = 0;
#pragma unroll
      for (int m = 0; m < 8; m++) {
        if (m >= nm) break;
        const bool near = (nmask >> m) & 1u;
        const unsigned long long bal = __ballot(near);
        const int rk = __builtin_amdgcn_mbcnt_hi((unsigned)(bal >> 32),
                                                 __builtin_amdgcn_mbcnt_lo((unsigned)bal, 0u));
        int before = 0, mt = 0;
#pragma unroll
        for (int w2 = 0; w2 < NWV; w2++) {
          const int k = cnt[m * NWV + w2];
          before += w2 < wv ? k : 0;
          mt += k;
        }
        if (near) E.nearl[total + before + rk] = (uint16_t)(lane + m * L);
        total += mt;
      }
      nwork = total;
      esync<L>();
#ifdef BX_MSTAMPS
      ms_acc[12] += (unsigned long long)nwork;
      ms_acc[13] += 1ull;
#endif
    }
    BX_MSTAMP(11);
    // Collider.position_apply (colliders.py:198-240), first the contacts of
    // the work rows (contact_gen); the pass's Info rows are written here. A
    // row that does not penetrate has exact-zero impulses in both passes (its
    // `c < 0` / `penetration > 0` masks, colliders.py:332, 437): only the
    // penetrating (or NaN) rows are listed, in (m, wave, lane) order, with
    // their contacts (E.cbuf / the overflow slice) and their compact index in
    // E.sidx
    int nstore = 0;
    for (int m0 = 0, par = 0; m0 < nwork; m0 += L, par ^= 1) {
      const int x = m0 + lane;
      const bool has = x < nwork;
      const int r = has ? (bph ? (int)E.nearl[x] : BX_MULTI_RX(x)) : 0;
      v3 cp = mk(0.f, 0.f, 0.f), cn = mk(0.f, 0.f, 0.f);
      float pen = 0.f;
      bool st = false;
      if (has) {
        RowC R = row_from_lds(E, r);
        QP a = ldqp(E.qp + R.a * QP_STRIDE), b = ldqp(E.qp + R.b * QP_STRIDE);
        v3 cvel;
        contact_gen<F>(R, a, b, cp, cvel, cn, pen);
        st = pen > 0.f || is_nan(pen);
        // Info contact rows of the last position pass (system.py:36-43)
        if (last && valid && info_rows) {
          if (io.pos) st3(io.pos + x * 3, cp);
          if (io.normal) st3(io.normal + x * 3, cn);
          if (io.pen) io.pen[x] = pen;
          if (io.cell) io.cell[x] = c.i(H.o_row + r * ROW_STRIDE + R_FLAT);
        }
      }
      const unsigned long long bal = __ballot(st);
      const int rk = __builtin_amdgcn_mbcnt_hi((unsigned)(bal >> 32),
                                               __builtin_amdgcn_mbcnt_lo((unsigned)bal, 0u));
      // (two count buffers: a wave may write the next iteration's counts
      // while another still reads these)
      int* cnt = E.nearc + 32 + par * NWV;
      if ((lane & 63) == 0) cnt[wv] = __popcll(bal);
      esync<L>();
      int before = 0, tot = 0;
#pragma unroll
      for (int w2 = 0; w2 < NWV; w2++) {
        const int k = cnt[w2];
        before += w2 < wv ? k : 0;
        tot += k;
      }
      if (st) {
        const int y = nstore + before + rk;
        float* d = cb_at(y);
        if (y < MCBUF) {
          st4a(d, f32x4{cp.x, cp.y, cp.z, cn.x});
          st4a(d + 4, f32x4{cn.y, cn.z, pen, 0.f});
          cbrow[y] = (uint16_t)r;
        } else {
          d[0] = cp.x; d[1] = cp.y; d[2] = cp.z; d[3] = cn.x;
          d[4] = cn.y; d[5] = cn.z; d[6] = pen; d[8] = __int_as_float(r);
        }
        E.sidx[r] = (uint16_t)y;
      }
      nstore += tot;
    }
    esync<L>();
#ifdef BX_MSTAMPS
    if (H.n_nn == 0) ms_acc[14] += (unsigned long long)nstore;
#endif
    BX_MSTAMP(4);
    // the position impulses of the listed rows, MCAP at a time: row y's sides
    // into the chunk's slots, then the tasks add the chunk
    const int nch = (nstore + MCAP - 1) / MCAP;
    for (int ch = 0; ch < nch; ch++) {
      const int y = ch * MCAP + lane;
      if (lane < MCAP && y < nstore) {
        float* d = cb_at(y);
        const v3 cp = mk(d[0], d[1], d[2]), cn = mk(d[3], d[4], d[5]);
        const float pen = d[6];
        const int r = cb_row(y);
        RowC R = row_from_lds(E, r);
        v3 oap, obp;
        q4 oar, obr;
        float dl;
        if (is_nan(pen)) {
          // a NaN contact's impulses are NaN on both sides (the reference's
          // masked products, colliders.py:332-333: NaN * 0)
          const float pz = nan_of(pen);
          oap = obp = mk(pz, pz, pz);
          oar = obr = q4{pz, pz, pz, pz};
          dl = pz;
        } else {
          QP a = ldqp(E.qp + R.a * QP_STRIDE), b = ldqp(E.qp + R.b * QP_STRIDE);
          v3 pap, pbp;
          q4 par, pbr;
          float unused;
          ld_slot(E.prev + R.a * PREV_STRIDE, pap, par, unused);
          ld_slot(E.prev + R.b * PREV_STRIDE, pbp, pbr, unused);
          dl = position_contact<F, true>(R, a, b, pap, par, pbp, pbr, cp, cn, pen, oap, oar, obp, obr);
        }
        d[7] = dl;
        st_mslot(E.cslot + lane * MSLOT_STRIDE, oap, mk(oar.x, oar.y, oar.z));
        if (!is_oneway<F>(R.oneway)) st_mslot(E.cslot + (MCAP + lane) * MSLOT_STRIDE, obp, mk(obr.x, obr.y, obr.z));
      }
      // the zero task partial (the bodies' padding; the near list and the
      // NearNeighbors scratch share these words)
      if (ch == 0 && lane < TSLOT_STRIDE) E.tslot[H.T * TSLOT_STRIDE + lane] = 0.f;
      esync<L>();
      tasks(ch);
      esync<L>();
    }
    BX_MSTAMP(5);
    if (X.hasB) {
      v3 dp = mk(0.f, 0.f, 0.f), dl = mk(0.f, 0.f, 0.f);
      // (no listed row: every partial is zero, and 0 / (eps + 0) adds zeros)
      if (nstore > 0) body_combine(X.bt, E.tslot, 1e-6f, dp, dl);
      // the body's one quaternion product of its summed angular impulses
      const q4 dr = 0.5f * vec_quat_mul(mul(X.B.I, dl), q.rot);
      q.pos = q.pos + mul(dp, X.B.pm);
      q.rot = q4{q.rot.w + dr.w * X.B.qm.w, q.rot.x + dr.x * X.B.qm.x, q.rot.y + dr.y * X.B.qm.y,
                 q.rot.z + dr.z * X.B.qm.z};
      st_rb(E.rb + lane * RB_STRIDE, q.pos, q.vel, q.ang);
      vproj(q, ppos, prot, X.B, h, false, true);
      stqp(myqp, q);
    }
    esync<L>();
    BX_MSTAMP(6);
    // Collider.velocity_apply (colliders.py:155-196): the listed rows
    for (int ch = 0; ch < nch; ch++) {
      const int y = ch * MCAP + lane;
      if (lane < MCAP && y < nstore) {
        const float* d = cb_at(y);
        const v3 cp = mk(d[0], d[1], d[2]), cn = mk(d[3], d[4], d[5]);
        const float pen = d[6], dl = d[7];
        const int r = cb_row(y);
        RowC R = row_from_lds(E, r);
        v3 oav, oaa, obv, oba;
        if (is_nan(pen)) {
          const float pz = nan_of(pen);
          oav = oaa = obv = oba = mk(pz, pz, pz);
        } else {
          QP a = ldqp(E.qp + R.a * QP_STRIDE), b = ldqp(E.qp + R.b * QP_STRIDE);
          v3 rap, rav, raa, rbp, rbv, rba;
          ld_rb(E.rb + R.a * RB_STRIDE, rap, rav, raa);
          ld_rb(E.rb + R.b * RB_STRIDE, rbp, rbv, rba);
          velocity_contact<F>(R, h, a, b, rap, rav, raa, rbp, rbv, rba, cp, cn, pen, dl, oav, oaa, obv,
                              oba);
        }
        st_mslot(E.cslot + lane * MSLOT_STRIDE, oav, oaa);
        if (!is_oneway<F>(R.oneway)) st_mslot(E.cslot + (MCAP + lane) * MSLOT_STRIDE, obv, oba);
      }
      esync<L>();
      tasks(ch);
      esync<L>();
    }
    BX_MSTAMP(7);
    if (X.hasB) {
      v3 dv = mk(0.f, 0.f, 0.f), dav = mk(0.f, 0.f, 0.f);
      if (nstore > 0) body_combine(X.bt, E.tslot, 1e-6f, dv, dav);
      q.vel = mul(q.vel + dv, X.B.pm);
      q.ang = mul(q.ang + dav, X.B.rm);
      stqp(myqp, q);
      icv = icv + dv;
      ica = ica + dav;
      iaa = iaa + dpa_last;
    }
    // the listed rows leave the index (the next pass's listing writes it
    // after its barriers)
    for (int y = lane; y < nstore; y += L) E.sidx[cb_row(y)] = (uint16_t)0xFFFFu;
    esync<L>();
    BX_MSTAMP(8);
  }
  // (the Info accumulators alias the contact slots, dead from here)
  if (X.hasB) {
    float* acc = E.acc + lane * ACC_STRIDE;
    st3(acc + ACC_ICV, icv);
    st3(acc + ACC_ICA, ica);
    st3(acc + ACC_IAA, iaa);
  }
  esync<L>();
  BX_MSTAMP(10);
#undef BX_MULTI_RX
#ifdef BX_MSTAMPS
  if (threadIdx.x == 0) {
#pragma unroll
    for (int k = 0; k < 15; k++) bx_mstamp_wave[blockIdx.x & 4095][k] += ms_acc[k];
    bx_mstamp_wave[blockIdx.x & 4095][15] += 1ull;
  }
#endif
}

// System._pbd_info contact part (system.py:327-340 -> Collider.apply): info
// contact (vel, ang) per body into acc[ACC_ICV], acc[ACC_ICA]
template <int L>
__device__ void pbd_info(const Cst& c, const BlobHdr& H, const Env& E, int lane) {
  const int N = H.N, Rn = H.R;
  // culled groups: the cells nearest in this qp (the reference's Info uses
  // whatever its stateful cull object last selected)
  if (H.n_nn) nn_select<L>(c, H, E, lane);
  for (int r = lane; r < Rn; r += L) {
    if (!row_active(H, E, r)) {
      zero_row_slots(c, H, E, r);
      continue;
    }
    RowC R = load_row(c, H, r);
    QP a = ldqp(E.qp + R.a * QP_STRIDE), b = ldqp(E.qp + R.b * QP_STRIDE);
    v3 cpos, cvel, n;
    float pen;
    contact_gen_x<F_GEN>(c, H, r, R, a, b, cpos, cvel, n, pen);
    v3 oav, oaa, obv, oba;
    impulse_contact<F_GEN>(R, a, b, cpos, cvel, n, pen, oav, oaa, obv, oba);
    float* sa = E.cslot + r * SLOT_STRIDE;
    float* sb = E.cslot + (E.nR + r) * SLOT_STRIDE;
    st3(sa, oav); st3(sa + 3, oaa);
    sa[7] = nonzero3(oav);
    st3(sb, obv); st3(sb + 3, oba);
    sb[7] = nonzero3(obv);
  }
  esync<L>();
  for (int b = lane; b < N; b += L) {
    v3 dv = mk(0.f, 0.f, 0.f), da = mk(0.f, 0.f, 0.f);
    int i = c.i(H.o_cl_off + b), e = c.i(H.o_cl_off + b + 1);
    while (i < e) {
      int g = c.i(H.o_cl + i) >> 24;
      v3 gv = mk(0.f, 0.f, 0.f), ga = mk(0.f, 0.f, 0.f);
      float cnt = 0.f;
      for (; i < e && (c.i(H.o_cl + i) >> 24) == g; i++) {
        const float* s = E.cslot + (c.i(H.o_cl + i) & 0xFFFFFF) * SLOT_STRIDE;
        gv = gv + ld3(s);
        ga = ga + ld3(s + 3);
        cnt += s[7];
      }
      float d = 1e-8f + cnt;
      dv = dv + gv / d;
      da = da + ga / d;
    }
    float* acc = E.acc + b * ACC_STRIDE;
    st3(acc + ACC_ICV, dv);
    st3(acc + ACC_ICA, da);
  }
  esync<L>();
}

// ---------------------------------------------------------------------------
// env layer (ant.py:222-282, half_cheetah.py:178-214, humanoid.py:246-338)
// ---------------------------------------------------------------------------

// joint angles and velocities into E.ang (Joint.angle_vel, joints.py:197-226)
// hj: the lane's register-hoisted joint (SINGLE mode, J <= L: joint j ==
// lane), which spares the blob reloads on the observation path
template <int L>
__device__ void joint_angles(const Cst& c, const BlobHdr& H, const Env& E, int lane,
                             const JointC* hj = nullptr) {
  for (int j = lane; j < H.J; j += L) {
    JointC Jc = hj ? *hj : load_joint(c, H, j);
    QP p = ldqp(E.qp + Jc.bp * QP_STRIDE), q = ldqp(E.qp + Jc.bc * QP_STRIDE);
    v3 axes[3];
    float ang[3];
    axis_angle<F_ALL>(Jc, p, q, axes, ang);
    v3 dv = p.ang - q.ang;
#pragma unroll
    for (int l = 0; l < 3; l++) {
      if (l < Jc.n_angles) {
        E.ang[Jc.angle_off + l] = ang[l];
        E.ang[H.D + Jc.angle_off + l] = dot(dv, axes[l]);
      }
    }
  }
}

__device__ __forceinline__ float clip1(float x) { return clampn(x, -1.f, 1.f); }

// math.quat_to_euler(q)[2] (math.py:80-91) of a QP record's rot (w, x, y, z)
__device__ __forceinline__ float euler_z(const float* q) {
  return atan2f(-2.f * q[1] * q[2] + 2.f * q[0] * q[3],
                q[1] * q[1] + q[0] * q[0] - q[3] * q[3] - q[2] * q[2]);
}

// math.quat_to_euler(q)[1] (math.py:80-91): asin(clip(2 q1 q3 + 2 q0 q2))
// of a QP record's rot (w, x, y, z)
__device__ __forceinline__ float euler_y(const float* q) {
  return asinf(clampn(2.f * q[1] * q[3] + 2.f * q[0] * q[2], -1.f, 1.f));
}

// Humanoid center of mass over bodies [:-1] (humanoid.py:336-338) -> red[32..35]
// n16 (SINGLE mode: N <= 16): a fixed trip count, so the bodies' masses
// (uniform scalar loads) and qp reads issue together instead of one
// dependent load per body; same sum order, the masked tail adds 0 * pos,
// which leaves acc and m unchanged. (Not the lanes' hoisted masses through
// readlane: the call sits in a lane-0 branch, where a spilled mass is
// restored for the active lanes only.)
// lmass (the SINGLE kernels at 16 lanes): the bodies' masses staged in LDS
// once per launch (E.red + 16, from the lanes' hoisted records: the same
// bits), read there instead of from the blob
__device__ void humanoid_com(const Cst& c, const BlobHdr& H, const float* qp, v3& com, float& msum,
                             bool n16 = false, const float* lmass = nullptr) {
  v3 acc = mk(0.f, 0.f, 0.f);
  float m = 0.f;
  if (n16) {
#pragma unroll
    for (int b = 0; b < 16; b++) {
      const bool in = b < H.N - 1;
      const int bb = in ? b : 0;
      const float w = in ? (lmass ? lmass[bb] : c.f(H.o_body + bb * BODY_STRIDE + BODY_MASS)) : 0.f;
      acc = acc + w * ld3(qp + bb * QP_STRIDE);
      m += w;
    }
    com = acc / m;
    msum = m;
    return;
  }
  for (int b = 0; b < H.N - 1; b++) {
    float mb = c.f(H.o_body + b * BODY_STRIDE + BODY_MASS);
    acc = acc + mb * ld3(qp + b * QP_STRIDE);
    m += mb;
  }
  com = acc / m;
  msum = m;
}

// observation element i of the env kind
// env-program specialisation: the hot env kinds get step kernels holding
// only their own env code (EK_ANT, EK_HUM: Humanoid and HumanoidStandup,
// EK_CHEETAH: HalfCheetah); EK_ANY carries every kind, chosen at run time
// (EK_PUSHER: Pusher, round 6: its 50 substeps with the damping folded)
enum { EK_ANY = 0, EK_ANT = 1, EK_HUM = 2, EK_CHEETAH = 3, EK_PUSHER = 4 };
template <int EK>
__device__ __forceinline__ constexpr bool ek_has(int k) {
  return EK == EK_ANY || (EK == EK_ANT && k == BX_ENV_ANT) ||
         (EK == EK_HUM && (k == BX_ENV_HUMANOID || k == BX_ENV_HUMANOID_STANDUP)) ||
         (EK == EK_CHEETAH && k == BX_ENV_HALFCHEETAH) || (EK == EK_PUSHER && k == BX_ENV_PUSHER);
}
#define KIND_IS(k) (ek_has<EK>(k) && kind == (k))

// counter-based uniform: splitmix64 of (seed, global index) -> [lo, hi)
__device__ __forceinline__ float uniform_at(uint64_t seed, uint64_t i, float lo, float hi) {
  uint64_t z = seed * 0x9E3779B97F4A7C15ull + i + 0x632BE59BD9B4E019ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  z = z ^ (z >> 31);
  float u = (float)(z >> 40) * (1.0f / 16777216.0f);
  return lo + (hi - lo) * u;
}

// the arm tip of the reachers: body coef[1]'s (.11, 0, 0) in the world and
// its velocity (QP.to_world, base.py:112-126)
__device__ __forceinline__ void arm_tip(const Env& E, const float* coef, v3& tp, v3& tv) {
  const float* a = E.qp + (int)coef[1] * QP_STRIDE;
  v3 off = rotate(mk(.11f, 0.f, 0.f), q4{a[3], a[4], a[5], a[6]});
  tp = ld3(a) + off;
  tv = ld3(a + 7) + cross(ld3(a + 10), off);
}

template <int EK>
__device__ float obs_elem(const Cst& c, const BlobHdr& H, const Env& E, int kind, int flags, int i,
                          const float* act, int aw, bool valid, const float* coef) {
  const int N = H.N, D = H.D;
  const float* q0 = E.qp;
  // exclude_current_positions_from_observation=False: the torso's x (and y)
  // precede z (ant.py:262-265, humanoid.py:289-292, half_cheetah.py:206-209)
  const bool loco2d = KIND_IS(BX_ENV_HOPPER) || KIND_IS(BX_ENV_WALKER2D);
  if (flags & BX_OBS_XY) {
    if (KIND_IS(BX_ENV_HALFCHEETAH) || loco2d) {
      if (i == 0) return q0[0];
      i -= 1;
    } else {
      if (i < 2) return q0[i];
      i -= 2;
    }
  }
  if (KIND_IS(BX_ENV_ANT)) {
    if (i == 0) return q0[2];
    i -= 1;
    if (i < 4) return q0[3 + i];
    i -= 4;
    if (i < D) return E.ang[i];
    i -= D;
    if (i < 3) return q0[7 + i];
    i -= 3;
    if (i < 3) return q0[10 + i];
    i -= 3;
    if (i < D) return E.ang[D + i];
    i -= D;
    if (i < 3 * N) return clip1(E.acc[(i / 3) * ACC_STRIDE + ACC_ICV + i % 3]);
    i -= 3 * N;
    return clip1(E.acc[(i / 3) * ACC_STRIDE + ACC_ICA + i % 3]);
  }
  if (loco2d) {
    // hopper.py:231-246: [z, ang_y, joint angles, vel x, vel z, ang y, joint vels]
    if (i == 0) return q0[2];
    if (i == 1) return euler_y(q0 + 3);
    i -= 2;
    if (i < D) return E.ang[i];
    i -= D;
    if (i == 0) return q0[7];
    if (i == 1) return q0[9];
    if (i == 2) return q0[11];
    i -= 3;
    return E.ang[D + i];
  }
  if (KIND_IS(BX_ENV_INVERTED_PENDULUM)) {
    // [cart pos x, joint angles, cart vel x, joint vels]
    if (i == 0) return q0[0];
    i -= 1;
    if (i < D) return E.ang[i];
    i -= D;
    if (i == 0) return q0[7];
    return E.ang[D + i - 1];
  }
  if (KIND_IS(BX_ENV_INVERTED_DOUBLE_PENDULUM)) {
    // [cart pos x, sin(angles), cos(angles), cart vel x, joint vels]
    if (i == 0) return q0[0];
    i -= 1;
    if (i < D) return sinf(E.ang[i]);
    i -= D;
    if (i < D) return cosf(E.ang[i]);
    i -= D;
    if (i == 0) return q0[7];
    return E.ang[D + i - 1];
  }
  if (KIND_IS(BX_ENV_ACROBOT)) return E.ang[i];  // [joint angles, joint vels]
  if (KIND_IS(BX_ENV_REACHER) || KIND_IS(BX_ENV_REACHERANGLE)) {
    // reacher.py:205-224: [cos(angles), sin(angles), target xy, tip vel xy,
    // tip - target]; the tip is the arm body's (.11, 0, 0)
    if (i < D) return cosf(E.ang[i]);
    i -= D;
    if (i < D) return sinf(E.ang[i]);
    i -= D;
    const float* tq = E.qp + (int)coef[0] * QP_STRIDE;
    if (i < 2) return tq[i];
    i -= 2;
    v3 tp, tv;
    arm_tip(E, coef, tp, tv);
    if (i < 2) return i == 0 ? tv.x : tv.y;
    i -= 2;
    v3 d = tp - ld3(tq);
    return i == 0 ? d.x : (i == 1 ? d.y : d.z);
  }
  if (KIND_IS(BX_ENV_SWIMMER)) {
    // swimmer.py:257-272: [ang z, joint angles, vel x, vel y, ang z, joint vels]
    if (i == 0) return euler_z(q0 + 3);
    i -= 1;
    if (i < D) return E.ang[i];
    i -= D;
    if (i < 2) return q0[7 + i];
    if (i == 2) return q0[12];
    i -= 3;
    return E.ang[D + i];
  }
  if (KIND_IS(BX_ENV_UR5E) || KIND_IS(BX_ENV_FETCH)) {
    // ur5e.py:115-135 / fetch.py:101-121, egocentric in the torso's frame:
    // [torso fwd, torso up, |target|, target dir, local pos (N x 3), local
    // vel (N x 3), contact flags (N: |Info contact vel|^2 > 1e-5)]
    const float* t = E.qp + (int)coef[0] * QP_STRIDE;
    const q4 tr{t[3], t[4], t[5], t[6]};
    if (i < 3) { v3 f = rotate(mk(1.f, 0.f, 0.f), tr); return i == 0 ? f.x : (i == 1 ? f.y : f.z); }
    i -= 3;
    if (i < 3) { v3 u = rotate(mk(0.f, 0.f, 1.f), tr); return i == 0 ? u.x : (i == 1 ? u.y : u.z); }
    i -= 3;
    const q4 ti = quat_inv(tr);
    if (i < 4) {
      v3 tl = rotate(ld3(E.qp + (int)coef[1] * QP_STRIDE) - ld3(t), ti);
      float mag = norm(tl);
      if (i == 0) return mag;
      v3 d = tl / (1e-6f + mag);
      return i == 1 ? d.x : (i == 2 ? d.y : d.z);
    }
    i -= 4;
    if (i < 3 * N) {
      const int b = i / 3;
      v3 l = rotate(ld3(E.qp + b * QP_STRIDE) - ld3(t), ti);
      return i % 3 == 0 ? l.x : (i % 3 == 1 ? l.y : l.z);
    }
    i -= 3 * N;
    if (i < 3 * N) {
      const int b = i / 3;
      v3 l = rotate(ld3(E.qp + b * QP_STRIDE + 7), ti);
      return i % 3 == 0 ? l.x : (i % 3 == 1 ? l.y : l.z);
    }
    i -= 3 * N;
    const float* cv = E.acc + i * ACC_STRIDE + ACC_ICV;
    return cv[0] * cv[0] + cv[1] * cv[1] + cv[2] * cv[2] > 0.00001f ? 1.f : 0.f;
  }
  if (KIND_IS(BX_ENV_GRASP)) {
    // grasp.py:132-175, in the palm's frame: [|object|, object dir, |target|,
    // target dir, local pos (N x 3), local vel (N x 3), hand to object, hand
    // vel, heading to object, |object to target|, its dir, object heading,
    // contact flags (N)]
    const int pi = (int)coef[0], oi = (int)coef[1], gi = (int)coef[2], hi = (int)coef[3];
    const float* pq = E.qp + pi * QP_STRIDE;
    const q4 ri = quat_inv(q4{pq[3], pq[4], pq[5], pq[6]});
    if (i < 8) {
      const int b = i < 4 ? oi : gi;
      v3 l = rotate(ld3(E.qp + b * QP_STRIDE) - ld3(pq), ri);
      float mag = norm(l);
      const int k = i % 4;
      if (k == 0) return mag;
      v3 dd = l / (1e-6f + mag);
      return k == 1 ? dd.x : (k == 2 ? dd.y : dd.z);
    }
    i -= 8;
    if (i < 3 * N) {
      v3 l = rotate(ld3(E.qp + (i / 3) * QP_STRIDE) - ld3(pq), ri);
      return i % 3 == 0 ? l.x : (i % 3 == 1 ? l.y : l.z);
    }
    i -= 3 * N;
    if (i < 3 * N) {
      v3 l = rotate(ld3(E.qp + (i / 3) * QP_STRIDE + 7), ri);
      return i % 3 == 0 ? l.x : (i % 3 == 1 ? l.y : l.z);
    }
    i -= 3 * N;
    v3 h2o = ld3(E.qp + oi * QP_STRIDE) - ld3(pq);
    v3 hv = ld3(E.qp + hi * QP_STRIDE + 7);
    if (i < 3) return i == 0 ? h2o.x : (i == 1 ? h2o.y : h2o.z);
    i -= 3;
    if (i < 3) return i == 0 ? hv.x : (i == 1 ? hv.y : hv.z);
    i -= 3;
    if (i == 0) return dot(h2o / (1e-6f + norm(h2o)), hv);
    i -= 1;
    v3 o2t = ld3(E.qp + gi * QP_STRIDE) - ld3(E.qp + oi * QP_STRIDE);
    float om = norm(o2t);
    v3 od = o2t / (1e-6f + om);
    if (i == 0) return om;
    i -= 1;
    if (i < 3) return i == 0 ? od.x : (i == 1 ? od.y : od.z);
    i -= 3;
    if (i == 0) return dot(od, ld3(E.qp + oi * QP_STRIDE + 7));
    i -= 1;
    const float* cv = E.acc + i * ACC_STRIDE + ACC_ICV;
    return cv[0] * cv[0] + cv[1] * cv[1] + cv[2] * cv[2] > 0.00001f ? 1.f : 0.f;
  }
  if (KIND_IS(BX_ENV_PUSHER)) {
    // pusher.py:232-242: [joint angles, joint vels, tip, object, goal positions]
    if (i < 2 * D) return E.ang[i];
    i -= 2 * D;
    const int b = (int)coef[i / 3];
    return E.qp[b * QP_STRIDE + i % 3];
  }
  if (KIND_IS(BX_ENV_HALFCHEETAH)) {
    if (i == 0) return q0[2];
    if (i == 1) return q0[3];
    if (i == 2) return q0[5];
    i -= 3;
    if (i < D) return E.ang[i];
    i -= D;
    if (i == 0) return q0[7];
    if (i == 1) return q0[9];
    if (i == 2) return q0[11];
    i -= 3;
    return E.ang[D + i];
  }
  // humanoid
  if (i == 0) return q0[2];
  i -= 1;
  if (i < 4) return q0[3 + i];
  i -= 4;
  if (i < D) return E.ang[i];
  i -= D;
  if (i < 3) return q0[7 + i];
  i -= 3;
  if (i < 3) return q0[10 + i];
  i -= 3;
  if (i < D) return E.ang[D + i];
  i -= D;
  v3 com = ld3(E.red + 32);
  float msum = E.red[35];
  int M = N - 1;
  if (i < 9 * M) {
    int b = i / 9, rc = i % 9, r = rc / 3, cc = rc % 3;
    float mb = c.f(H.o_body + b * BODY_STRIDE + BODY_MASS);
    v3 d = ld3(E.qp + b * QP_STRIDE) - com;
    float nn = norm(d);
    float v = mb * (float)(r == cc) * (nn * nn);
    float dr = r == 0 ? d.x : (r == 1 ? d.y : d.z);
    float dc = cc == 0 ? d.x : (cc == 1 ? d.y : d.z);
    float Ir = c.f(H.o_body + b * BODY_STRIDE + BODY_I + r);
    v += (r == cc ? Ir : 0.f) - dr * dc;
    return v;
  }
  i -= 9 * M;
  if (i < 3 * M) {
    int b = i / 3, k = i % 3;
    float mb = c.f(H.o_body + b * BODY_STRIDE + BODY_MASS);
    return mb * E.qp[b * QP_STRIDE + 7 + k] / msum;
  }
  i -= 3 * M;
  if (i < 3 * M) {
    int b = i / 3, k = i % 3;
    v3 d = ld3(E.qp + b * QP_STRIDE) - com;
    v3 cr = cross(d, ld3(E.qp + b * QP_STRIDE + 7));
    float nn = norm(d);
    float v = k == 0 ? cr.x : (k == 1 ? cr.y : cr.z);
    return v / (1e-7f + nn * nn);
  }
  i -= 3 * M;
  // qfrc_actuator: unmasked take (index -1 clips to 0), times strength
  for (int a = 0; a < H.K; a++) {
    ActC A = load_act(c, H, a);
    int dof = c.i(H.o_joint + A.joint * JOINT_STRIDE + J_DOF);
    if (i < dof) {
      // constant indices into A.idx (a dynamic one would put A on the stack)
      const int ix = i == 0 ? A.idx[0] : (i == 1 ? A.idx[1] : A.idx[2]);
      return (valid ? act[take_idx(ix, aw)] : 0.f) * A.strength;
    }
    i -= dof;
  }
  return 0.f;
}

// obs_out null: nothing written (an env past the batch); act null: the
// action reads as zeros (reset's _get_obs(qp, info, jp.zeros(action_size)))
template <int L, int EK = EK_ANY>
__device__ void env_observe(const Cst& c, const BlobHdr& H, const Env& E, int lane, int kind,
                            int flags, int obs_size, const float* act, int aw, float* obs_out,
                            const float* coef, const JointC* hj = nullptr,
                            const BodyC* hbody = nullptr, const ActC* hact = nullptr) {
#if defined(BX_OSTAMPS) && defined(BX_TU_FAST)
  // (diagnostic: the observation's parts into stamp slots 5..9)
  unsigned long long ost_last;
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(ost_last)::"memory");
#define BX_OST(k)                                                                  \
  do {                                                                             \
    __builtin_amdgcn_sched_barrier(0);                                             \
    unsigned long long _t;                                                         \
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(_t)::"memory");     \
    __builtin_amdgcn_sched_barrier(0);                                             \
    if (threadIdx.x == 0) bx_stamp_wave[blockIdx.x & 4095][k] += _t - ost_last;    \
    ost_last = _t;                                                                 \
  } while (0)
#else
#define BX_OST(k) do {} while (0)
#endif
  joint_angles<L>(c, H, E, lane, hj);
  BX_OST(0);
  if ((KIND_IS(BX_ENV_HUMANOID) || KIND_IS(BX_ENV_HUMANOID_STANDUP)) && lane == 0) {
    v3 com;
    float msum;
    humanoid_com(c, H, E.qp, com, msum, L == 16 && hbody != nullptr,
                 L == 16 && hbody != nullptr ? E.red + 16 : nullptr);
    st3(E.red + 32, com);
    E.red[35] = msum;
  }
  esync<L>();
  BX_OST(1);
  if (!obs_out) return;
  if constexpr (EK == EK_ANT) {
    // the Ant observation (ant.py:257-282) written lane by lane without the
    // per-element branch chain: lane l holds torso scalar l, joint l's angle
    // and velocity, and body l's clipped contact vel / ang
    const int N = H.N, D = H.D;
    const int x = (flags & BX_OBS_XY) ? 2 : 0;
    const float* q0 = E.qp;
    for (int l = lane; l < x + 11; l += L) {
      // (x, y,) z, rot 4 | vel 3, ang 3
      const int k = l - x;
      float v = l < x ? q0[l] : (k < 5 ? q0[2 + k] : q0[7 + (k - 5)]);
      obs_out[k < 5 ? l : x + 5 + D + (k - 5)] = v;
    }
    for (int j = lane; j < D; j += L) {
      obs_out[x + 5 + j] = E.ang[j];
      obs_out[x + 11 + D + j] = E.ang[D + j];
    }
    if (coef[7] != 0.f)  // use_contact_forces
      for (int b = lane; b < N; b += L) {
        const float* a = E.acc + b * ACC_STRIDE;
        float* o = obs_out + x + 11 + 2 * D + 3 * b;
#pragma unroll
        for (int k = 0; k < 3; k++) {
          o[k] = clip1(a[ACC_ICV + k]);
          o[3 * N + k] = clip1(a[ACC_ICA + k]);
        }
      }
    return;
  }
  if constexpr (EK == EK_HUM && L <= 64) {
    // the Humanoid / HumanoidStandup observation (humanoid.py:282-334) lane
    // by lane: torso scalars and joints as Ant's, then lane b writes body b's
    // cinert (9), com velocity (3) and com angular term (3), and lane a its
    // actuator's qfrc entries at the exclusive prefix sum of the dofs
    const int N = H.N, D = H.D, M = N - 1;
    const int x = (flags & BX_OBS_XY) ? 2 : 0;
    const float* q0 = E.qp;
    for (int l = lane; l < x + 11; l += L) {
      const int k = l - x;
      float v = l < x ? q0[l] : (k < 5 ? q0[2 + k] : q0[7 + (k - 5)]);
      obs_out[k < 5 ? l : x + 5 + D + (k - 5)] = v;
    }
    for (int j = lane; j < D; j += L) {
      obs_out[x + 5 + j] = E.ang[j];
      obs_out[x + 11 + D + j] = E.ang[D + j];
    }
    const int base = x + 11 + 2 * D;
    const v3 com = ld3(E.red + 32);
    const float msum = E.red[35];
    BX_OST(2);
    for (int b = lane; b < M; b += L) {
      // SINGLE mode: body b is the lane's, its constants hoisted (hbody)
      const int ob = H.o_body + b * BODY_STRIDE;
      const float mb = hbody ? hbody->mass : c.f(ob + BODY_MASS);
      const float Ia[3] = {hbody ? hbody->I.x : c.f(ob + BODY_I),
                           hbody ? hbody->I.y : c.f(ob + BODY_I + 1),
                           hbody ? hbody->I.z : c.f(ob + BODY_I + 2)};
      const v3 d = ld3(E.qp + b * QP_STRIDE) - com;
      const v3 vb = ld3(E.qp + b * QP_STRIDE + 7);
      const float nn = norm(d);
      const float dd[3] = {d.x, d.y, d.z};
      float* o = obs_out + base + 9 * b;
#pragma unroll
      for (int r = 0; r < 3; r++)
#pragma unroll
        for (int cc = 0; cc < 3; cc++) {
          float v = mb * (float)(r == cc) * (nn * nn);
          v += (r == cc ? Ia[r] : 0.f) - dd[r] * dd[cc];
          o[3 * r + cc] = v;
        }
      float* ov = obs_out + base + 9 * M + 3 * b;
      ov[0] = mb * vb.x / msum;
      ov[1] = mb * vb.y / msum;
      ov[2] = mb * vb.z / msum;
      const v3 cr = cross(d, vb);
      const float den = 1e-7f + nn * nn;
      float* oa = obs_out + base + 12 * M + 3 * b;
      oa[0] = cr.x / den;
      oa[1] = cr.y / den;
      oa[2] = cr.z / den;
    }
    BX_OST(3);
    // qfrc_actuator: unmasked take (index -1 clips to 0), times strength
    const bool ha = lane < H.K;
    ActC A{};
    int dof = 0;
    if (ha && hact && hj) {
      // the lane's hoisted actuator and joint (act_same: actuator a drives joint a)
      A = *hact;
      dof = hj->dof;
    } else if (ha) {
      A = load_act(c, H, lane);
      dof = c.i(H.o_joint + A.joint * JOINT_STRIDE + J_DOF);
    }
    int off = dof;  // inclusive scan over the env's lanes
    constexpr int W = L < 64 ? L : 64;
#pragma unroll
    for (int sh = 1; sh < W; sh <<= 1) {
      int t = __shfl_up(off, sh, W);
      if ((lane % W) >= sh) off += t;
    }
    off -= dof;
    float* oq = obs_out + base + 15 * M + off;
    // constant indices into A.idx (a dynamic one would put A on the stack)
#pragma unroll
    for (int i = 0; i < 3; i++)
      // (the row as staged in LDS for the physics: the same words, no second
      // read of the action row from HBM)
      if (i < dof) oq[i] = (act ? E.arow[take_idx(A.idx[i], aw)] : 0.f) * A.strength;
    BX_OST(4);
    return;
  }
  for (int i = lane; i < obs_size; i += L)
    obs_out[i] = obs_elem<EK>(c, H, E, kind, flags, i, act, aw, act != nullptr, coef);
}

// ---------------------------------------------------------------------------
// kernels
// ---------------------------------------------------------------------------



// kernel variants: MODE_GLOBAL (constants read from the HBM blob inside the
// loops), MODE_SINGLE (constants hoisted to registers), MODE_LDS (the blob's
// constant part copied to LDS once per workgroup, read there inside the loops)
enum { MODE_GLOBAL = 0, MODE_SINGLE = 1, MODE_LDS = 2, MODE_MULTI = 3 };

// step kernels: optional register-budget hint (A/B knob, BX_WAVES1)
#if defined(BX_WAVES1)
#define BX_STEP_ATTR __attribute__((amdgpu_waves_per_eu(1, 1)))
#else
#define BX_STEP_ATTR
#endif

// copies the constant blob into LDS (MODE_LDS); returns the env-area base
template <int MODE>
__device__ __forceinline__ float* stage_constants(const uint32_t* blob, const BlobHdr& H,
                                                  float* smem, Cst& c) {
  if constexpr (MODE == MODE_LDS) {
    uint32_t* cl = reinterpret_cast<uint32_t*>(smem);
    for (int i = threadIdx.x; i < H.const_words; i += blockDim.x) cl[i] = blob[i];
    __syncthreads();
    c.w = cl;
    return smem + H.const_words;
  } else {
    c.w = blob;
    return smem;
  }
}

template <int L, int MODE, int F, int M>
__device__ __forceinline__ void system_step_body(const StepArgs& A) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  BlobHdr H = *reinterpret_cast<const BlobHdr*>(A.blob);
  Cst c{A.blob};
  float* ebase = stage_constants<MODE>(A.blob, H, smem, c);
  constexpr bool S = MODE == MODE_SINGLE;
  constexpr bool MU = MODE == MODE_MULTI;
  // (MULTI: one env per workgroup of L threads, so the env's LDS base is
  // uniform by construction)
  const int lane = MU ? (int)threadIdx.x : (int)(threadIdx.x % L);
  const int le = MU ? 0 : (int)(threadIdx.x / L);
  const int64_t e = (int64_t)blockIdx.x * (MU ? 1 : (blockDim.x / L)) + le;
  const bool valid = e < A.n_envs;
  Env E = carve(ebase + le * H.env_words, H, MU);
  zero_slots(E, H, lane);
  // SINGLE: the lane image's loads go out before the state's
  Hoist<M, cl_width<F, M>()> X;
  if constexpr (S) {
    load_hoist<M, (F & F_JH) != 0, (F & F_R2) != 0, cl_width<F, M>()>(A.blob + H.o_lane, H, lane, X);
    stage_lim<L, F>(A.blob + H.o_lane, H, E, lane);
  }
  for (int b = lane; b < H.N; b += L) {
    if (valid) {
      load_qp_global(A.qin, e, b, E.qp + b * QP_STRIDE);
    } else {
      float* s = E.qp + b * QP_STRIDE;
      for (int k = 0; k < 13; k++) s[k] = k == 3 ? 1.f : 0.f;
    }
  }
  esync<L>();
  if constexpr (MU) {
    HoistM X;
    load_hoist_multi<L, (F & F_JH) != 0>(c, H, lane, X);
    // the broad phase's / NearNeighbors' constants into LDS, read by every pass
    if (H.o_bimg != 0) {
      const uint32_t* bg = c.w + H.o_bimg;
      for (int k = lane; k < BI_WORDS * H.R; k += L) E.bimg[k] = bg[k];
      const uint4* cg = reinterpret_cast<const uint4*>(c.w + H.o_cen);
      for (int k = lane; k < 2 * H.n_cen + H.n_mat + H.N; k += L) E.cen[k] = cg[k];
    }
    // no row has a compact contact index yet (row R: the tasks' padding)
    for (int r = lane; r <= H.R; r += L) E.sidx[r] = (uint16_t)0xFFFFu;
    // lane k's first read (place_centres: E.cen[2k]) is another wave's
    // write: no pass reads the tables before every wave has staged them
    esync<L>();
    const int64_t ro = valid ? e * H.info_rows : 0;
    RowInfoOut io{A.info.contact_pos ? A.info.contact_pos + ro * 3 : nullptr,
                  A.info.contact_normal ? A.info.contact_normal + ro * 3 : nullptr,
                  A.info.contact_penetration ? A.info.contact_penetration + ro : nullptr,
                  A.info.contact_cell ? A.info.contact_cell + ro : nullptr};
    pbd_step_multi<L, F>(c, H, E, lane, valid, valid ? A.act + e * A.act_stride : nullptr,
                         (int)A.act_width, X, io,
                         A.movf ? A.movf + (valid ? e : 0) * (int64_t)(H.R - MCBUF) * MOVF_W : nullptr);
  } else if constexpr (S) {
    v3 icv, ica, iaa;
    pbd_step_single<L, F, M>(c, H, E, lane, valid, valid ? A.act + e * A.act_stride : nullptr,
                             (int)A.act_width, X, icv, ica,
                       iaa);
  } else if (H.spring) {
    spring_step<L, F>(c, H, E, lane, valid, valid ? A.act + e * A.act_stride : nullptr, (int)A.act_width);
  } else {
    pbd_step<L, F>(c, H, E, lane, valid, valid ? A.act + e * A.act_stride : nullptr, (int)A.act_width);
  }
  if (!valid) return;
  for (int b = lane; b < H.N; b += L) {
    store_qp_global(A.qout, e, b, E.qp + b * QP_STRIDE);
    const float* acc = E.acc + b * ACC_STRIDE;
    const bx_info& I = A.info;
    if (I.contact_vel.ptr) {
      float* p = I.contact_vel.ptr + e * I.contact_vel.env_stride + b * I.contact_vel.body_stride;
      p[0] = acc[ACC_ICV]; p[1] = acc[ACC_ICV + 1]; p[2] = acc[ACC_ICV + 2];
    }
    if (I.contact_ang.ptr) {
      float* p = I.contact_ang.ptr + e * I.contact_ang.env_stride + b * I.contact_ang.body_stride;
      p[0] = acc[ACC_ICA]; p[1] = acc[ACC_ICA + 1]; p[2] = acc[ACC_ICA + 2];
    }
    if (I.actuator_vel.ptr) {
      float* p = I.actuator_vel.ptr + e * I.actuator_vel.env_stride + b * I.actuator_vel.body_stride;
      p[0] = 0.f; p[1] = 0.f; p[2] = 0.f;
    }
    if (I.actuator_ang.ptr) {
      float* p = I.actuator_ang.ptr + e * I.actuator_ang.env_stride + b * I.actuator_ang.body_stride;
      p[0] = acc[ACC_IAA]; p[1] = acc[ACC_IAA + 1]; p[2] = acc[ACC_IAA + 2];
    }
    // Info.joint: the spring step's accumulated dp_j; zero_info under pbd
    const float* ij = E.rb + b * RB_STRIDE;
    if (I.joint_vel.ptr) {
      float* p = I.joint_vel.ptr + e * I.joint_vel.env_stride + b * I.joint_vel.body_stride;
      for (int k = 0; k < 3; k++) p[k] = H.spring ? ij[k] : 0.f;
    }
    if (I.joint_ang.ptr) {
      float* p = I.joint_ang.ptr + e * I.joint_ang.env_stride + b * I.joint_ang.body_stride;
      for (int k = 0; k < 3; k++) p[k] = H.spring ? ij[3 + k] : 0.f;
    }
  }
  if constexpr (MU) return;  // MULTI wrote its Info rows from registers
  for (int r = lane; r < H.R; r += L) {
    const int x = row_info(c, H, E, r);
    if (x < 0) continue;
    const int64_t o = e * H.info_rows + x;
    const float* rd = E.rowd + r * ROWD_STRIDE;
    if (A.info.contact_pos) st3(A.info.contact_pos + o * 3, ld3(rd));
    if (A.info.contact_normal) st3(A.info.contact_normal + o * 3, ld3(rd + 3));
    if (A.info.contact_penetration) A.info.contact_penetration[o] = rd[6];
    if (A.info.contact_cell) A.info.contact_cell[o] = c.i(H.o_row + r * ROW_STRIDE + R_FLAT);
  }
}
template <int L, int MODE, int F, int M>
__global__ void __launch_bounds__(L > 64 ? L : 64) BX_STEP_ATTR system_step_kernel(StepArgs A) {
  system_step_body<L, MODE, F, M>(A);
}
// the MULTI kernel held to 256 registers per lane (VGPRs + AGPRs): two waves
// per SIMD. Past 256 (round 4: the row image's b-slot index took it to
// 256 + 4) one wave per SIMD fits and the CU holds half the envs: Ant
// Mountain(4) at 2,048 envs ran 1.8x slower (tools/multi_occ.py). At L = 128
// threads per env (two waves) four envs share a CU, when their LDS tail
// fits 40 KB (the compact contact slots, bx_capi.cpp)
template <int L, int JH = 0>
__global__ void __launch_bounds__(L) __attribute__((amdgpu_waves_per_eu(2)))
system_step_multi_kernel(StepArgs A) {
  system_step_body<L, MODE_MULTI, F_CC | F_TW | JH, 1>(A);
}



// Env.step fused with EpisodeWrapper/AutoResetWrapper (wrappers.py:105-148),
// for A.n_steps consecutive steps (bx_env_rollout_packed; 1 for bx_env_step):
// step t reads its action rows at act + t * act_step and writes its outputs at
// the output pointers + t * out_step (the rng stream at + t * rng_step); its
// input state is step t - 1's output, kept in LDS (the AutoReset select
// reloads first_qp there), so the lane image, the state and the per-env
// scalars are loaded once per launch, not once per step
// PK (the K-step rollout kernels, launched only on the packed layout of
// bx_env_rollout_packed / _random): step t's outputs are one block at
// out.qp.pos.ptr + t * out_step (qp (B, N, 16) | obs (B, O) | reward, done,
// steps, truncation (4, B) | metrics (B, M)), so the step derives every
// output pointer from that base instead of carrying eleven strided fields
// across the step loop (uniform registers the kernel otherwise spills)
// ONE (env_step_packed_kernel, launched for n_steps <= 1 only): one step,
// its first loads issued from the kernel arguments (EARLY below)
template <int L, int MODE, int F, int M, int EK = EK_ANY, bool PK = false, bool ONE = false>
__device__ __forceinline__ void env_step_body(const EnvArgs& A) {
  BX_KSTAMP_DECL
  extern __shared__ __attribute__((aligned(16))) float smem[];
  // the packed SINGLE-mode kernels (Env.step's bx_env_step_packed, the
  // rollouts) load the lane's state record first, from the kernel arguments
  // alone (the packed (B, N, 16) layout: in.qp.pos.env_stride = 16 N, no
  // blob header needed), so its HBM latency runs under the header / lane
  // image chain instead of after it
  constexpr bool EARLY = PK && ONE && MODE == MODE_SINGLE;
  f32x4 eq0 = {0.f, 0.f, 0.f, 0.f}, eq1 = eq0, eq2 = eq0;
  float eq3 = 0.f;
  if constexpr (EARLY) {
    const int64_t es = A.in.qp.pos.env_stride;
    const int nb = (int)(es >> 4);
    const int ln = (int)(threadIdx.x % L);
    const int64_t ee = (int64_t)blockIdx.x * (blockDim.x / L) + threadIdx.x / L;
    const float* qs = A.in.qp.pos.ptr + (ee < A.n_envs ? ee : 0) * es + (int64_t)(ln < nb ? ln : 0) * 16;
    eq0 = ld4a(qs);
    eq1 = ld4a(qs + 4);
    eq2 = ld4a(qs + 8);
    eq3 = qs[12];
  }
  // and the env's done / steps and the first action chunk (one element per
  // lane), likewise from the arguments alone
  float ed = 0.f, est = 0.f, ea0 = 0.f, ea1 = 0.f;
  if constexpr (EARLY) {
    const int ln = (int)(threadIdx.x % L);
    const int64_t ee = (int64_t)blockIdx.x * (blockDim.x / L) + threadIdx.x / L;
    const int64_t eel = ee < A.n_envs ? ee : 0;
    ed = A.in.done[eel];
    if (A.in.steps) est = A.in.steps[eel];
    const int aw0 = (int)A.act_width;
    constexpr int C0 = L < 64 ? L : 64;
    if (!A.draw && aw0 > 0 && ln < C0) {
      const float* ar = A.act + eel * A.act_stride;
      ea0 = ar[ln < aw0 ? ln : aw0 - 1];
      // (the second chunk too: Humanoid's 17-wide row)
      if (aw0 > C0) ea1 = ar[C0 + ln < aw0 ? C0 + ln : aw0 - 1];
    }
  }
  BlobHdr H = ONE ? A.hdr : *reinterpret_cast<const BlobHdr*>(A.blob);
  Cst c{A.blob};
  float* ebase = stage_constants<MODE>(A.blob, H, smem, c);
  constexpr bool S = MODE == MODE_SINGLE;
  const int lane = threadIdx.x % L;
  const int le = threadIdx.x / L;
  const int64_t e = (int64_t)blockIdx.x * (blockDim.x / L) + le;
  const bool valid = e < A.n_envs;
  // every load first, with clamped (unconditional) addresses so their
  // latencies overlap: the lane image (its address from the arguments, so
  // before the LDS setup that waits for the header), the per-env scalars,
  // the state and the first chunk of the action row; an invalid env's lanes
  // read env 0's (never stored)
  // (ONE: before the LDS setup, which waits for the header; the rollout
  // kernels keep the order their main loop was tuned with)
  Hoist<M, cl_width<F, M>()> X;
  // JB: the env-program kernels with joint halves (pbd_step_single's FOLD && JH)
  if constexpr (S && ONE)
    load_hoist<M, (F & F_JH) != 0, (F & F_R2) != 0, cl_width<F, M>(),
               (F & F_JH) != 0 && EK != EK_ANY && (F & F_C16) == 0>(A.lane_img, H, lane, X);
  Env E = carve(ebase + le * H.env_words, H);
  zero_slots(E, H, lane);
  BX_PSTAMP(5);
  const bx_env_params& P = A.P;
  const int kind = P.kind;
  const int aw = (int)A.act_width;
  const int64_t el = valid ? e : 0;
  if constexpr (S && !ONE)
    load_hoist<M, (F & F_JH) != 0, (F & F_R2) != 0, cl_width<F, M>(),
               (F & F_JH) != 0 && EK != EK_ANY && (F & F_C16) == 0>(A.blob + H.o_lane, H, lane, X);
  if constexpr (S) stage_lim<L, F>(ONE ? A.lane_img : A.blob + H.o_lane, H, E, lane);
  // the bodies' masses for humanoid_com (its lmass): lane b's hoisted body b
  // (the SINGLE kernels without body copies), into E.red + 16 once per launch
  if constexpr (S && L == 16 && !((F & F_JH) != 0 && EK != EK_ANY && (F & F_C16) == 0))
    E.red[16 + lane] = X.B.mass;
  BX_PSTAMP(6);
  // AutoResetWrapper.step: steps zeroed where the incoming done is set; done := 0
  float done_in = EARLY ? ed : A.in.done[el];
  float steps_in = EARLY ? est : (A.in.steps ? A.in.steps[el] : 0.f);
  if (!valid) done_in = steps_in = 0.f;
  // the target envs' per-env stream (advanced by one per env step)
  uint32_t rng_c = (A.in.rng && valid) ? A.in.rng[e] : 0u;
  constexpr int C = L < 64 ? L : 64;  // action-row chunk: one element per lane
  // on-device draws: the action row from the counter RNG, staged in LDS whole
  // (the host checks act_width <= act_read)
  const bool drw = A.draw != 0;
  auto draw_at = [&](int t, int i) {
    return uniform_at(A.draw_seed,
                      A.draw_offset + (uint64_t)t * A.draw_step + (uint64_t)el * (uint64_t)aw + (uint64_t)i,
                      A.draw_lo, A.draw_hi);
  };
  const float* arow_g = drw ? nullptr : A.act + el * A.act_stride;
  float a0 = 0.f;
  if (aw > 0 && lane < C) a0 = drw ? draw_at(0, lane < aw ? lane : aw - 1) : (EARLY ? ea0 : arow_g[lane < aw ? lane : aw - 1]);
  BX_PSTAMP(7);
  if constexpr (S) {
    // N <= L: the lane's body
    float qv[13];
    if constexpr (EARLY) {
#pragma unroll
      for (int k = 0; k < 4; k++) {
        qv[k] = eq0[k];
        qv[4 + k] = eq1[k];
        qv[8 + k] = eq2[k];
      }
      qv[12] = eq3;
    } else {
      load_qp_regs(A.in.qp, el, lane < H.N ? lane : 0, qv);
    }
    if (lane < H.N) {
      float* s = E.qp + lane * QP_STRIDE;
#pragma unroll
      for (int k = 0; k < 13; k++) s[k] = valid ? qv[k] : (k == 3 ? 1.f : 0.f);
    }
  } else {
    for (int b = lane; b < H.N; b += L) {
      if (valid) {
        load_qp_global(A.in.qp, e, b, E.qp + b * QP_STRIDE);
      } else {
        float* s = E.qp + b * QP_STRIDE;
        for (int k = 0; k < 13; k++) s[k] = k == 3 ? 1.f : 0.f;
      }
    }
  }
  BX_PSTAMP(8);
  const int nst = ONE ? 1 : (A.n_steps > 1 ? A.n_steps : 1);
  for (int t = 0; t < nst; t++) {
  // (draw mode: the env programs that read the raw row are refused on the
  // host; physics reads the staged row)
  const float* act = (valid && !drw) ? A.act + e * A.act_stride + t * A.act_step : nullptr;
  if (t > 0) {
    if (drw) {
      if (aw > 0 && lane < C) a0 = draw_at(t, lane < aw ? lane : aw - 1);
    } else {
      arow_g = A.act + el * A.act_stride + t * A.act_step;
      if (aw > 0 && lane < C) a0 = arow_g[lane < aw ? lane : aw - 1];
    }
  }
  // this step's outputs
  bx_env_state O;
  float* blk = nullptr;  // PK: this step's output block
  if constexpr (PK) {
    const int64_t B = A.n_envs;
    blk = A.out.qp.pos.ptr + t * A.out_step;
    O.obs = blk + B * H.N * 16;
    O.reward = O.obs + B * P.obs_size;
    O.done = O.reward + B;
    O.steps = O.reward + 2 * B;
    O.truncation = O.reward + 3 * B;
    O.metrics = P.n_metrics > 0 ? O.reward + 4 * B : nullptr;
    O.rng = A.out.rng ? A.out.rng + t * A.rng_step : nullptr;
  } else {
    O = A.out;
    if (t > 0) {
      const int64_t os = t * A.out_step;
      O.qp.pos.ptr += os; O.qp.rot.ptr += os; O.qp.vel.ptr += os; O.qp.ang.ptr += os;
      O.obs += os; O.reward += os; O.done += os;
      if (O.metrics) O.metrics += os;
      if (O.steps) O.steps += os;
      if (O.truncation) O.truncation += os;
      if (O.rng) O.rng += t * A.rng_step;
    }
  }
  // body b's output record
  auto store_out_qp = [&](int b, const float* src) {
    if constexpr (PK) {
      float* d = blk + (e * H.N + b) * 16;  // dword-aligned at any batch
      st4a(d, f32x4{src[0], src[1], src[2], src[3]});
      st4a(d + 4, f32x4{src[4], src[5], src[6], src[7]});
      st4a(d + 8, f32x4{src[8], src[9], src[10], src[11]});
      d[12] = src[12];
    } else {
      store_qp_global(O.qp, e, b, src);
    }
  };
  // the action row through LDS: its first act_read words stay staged (arow:
  // every index an actuator or force reads, jp.take clipping into the row),
  // and lane 0 sums the ctrl cost's squares in the reference's order (the
  // zero padding past the row adds exact zeros)
  float sq = 0.f;
  for (int i0 = 0; i0 < aw; i0 += C) {
    const int i = i0 + lane;
    float v = a0;
    if (i0 > 0 && lane < C)
      v = drw ? draw_at(t, i < aw ? i : aw - 1) : ((EARLY && i0 == C) ? ea1 : arow_g[i < aw ? i : aw - 1]);
    if (i >= aw || !valid) v = 0.f;
    if (drw && A.act_out && valid && lane < C && i < aw) A.act_out[((int64_t)t * A.n_envs + e) * aw + i] = v;
    if constexpr (EK == EK_ANT && L == 16) {
      // the Ant kernel: the squares summed across the env's 16 lanes by DPP
      // (a butterfly order instead of lane 0's serial one)
      if (i < H.act_read) E.arow[i] = v;
      sq += row_sum16(v * v);
      continue;
    }
    if (lane < C) {
      E.red[lane] = v;
      if (i < H.act_read) E.arow[i] = v;
    }
    esync<L>();
    if (lane == 0) {
#pragma unroll
      for (int k = 0; k < C; k++) sq += E.red[k] * E.red[k];
    }
    esync<L>();
  }
  esync<L>();
  float steps = 0.f;
  if (valid && (A.in.steps || t > 0)) steps = (P.auto_reset && done_in != 0.f) ? 0.f : steps_in;
  float done = P.auto_reset ? 0.f : done_in;
  float reward_sum = 0.f;
  const int reps = P.episode_length > 0 ? (P.action_repeat > 0 ? P.action_repeat : 1) : 1;
  BX_KSTAMP(10);
  v3 icv = mk(0.f, 0.f, 0.f);  // SINGLE: the lane's body's contact impulse sum
  for (int rep = 0; rep < reps; rep++) {
    v3 pos0 = ld3(E.qp);  // torso position before the step
    v3 com0 = mk(0.f, 0.f, 0.f);
    float msum = 0.f;
    if (KIND_IS(BX_ENV_HUMANOID) || KIND_IS(BX_ENV_SWIMMER))
      humanoid_com(c, H, E.qp, com0, msum, S && EK == EK_HUM && (F & F_JH) == 0,
                   S && L == 16 && EK == EK_HUM && (F & F_JH) == 0 ? E.red + 16 : nullptr);
    // the target envs' torso before the step (red words 36..38)
    if ((KIND_IS(BX_ENV_UR5E) || KIND_IS(BX_ENV_FETCH)) && lane == 0)
      st3(E.red + 36, ld3(E.qp + (int)P.coef[0] * QP_STRIDE));
    // Pusher's rewards come from the state before the step (pusher.py:212-217)
    float near0 = 0.f, dist0 = 0.f;
    if (KIND_IS(BX_ENV_PUSHER)) {
      v3 tip = ld3(E.qp + (int)P.coef[0] * QP_STRIDE), obj = ld3(E.qp + (int)P.coef[1] * QP_STRIDE);
      v3 goal = ld3(E.qp + (int)P.coef[2] * QP_STRIDE);
      near0 = -norm(obj - tip);
      dist0 = -norm(obj - goal);
    }
    // the action System.step reads: the env's own (staged in E.arow), or its
    // pre-step program's output (E.xact)
    const float* sact = valid ? E.arow : nullptr;
    int saw = aw;
    float* xact = E.xact;
    if (KIND_IS(BX_ENV_REACHERANGLE)) {
      // reacherangle.py:79: min + range * (a + 1) / 2 onto the angle limits
      if (valid && lane < aw) xact[lane] = P.coef[2 + lane] + P.coef[4 + lane] * ((act[lane] + 1.f) / 2.f);
      sact = valid ? xact : nullptr;
    } else if (KIND_IS(BX_ENV_SWIMMER)) {
      // swimmer.py:246-255: viscous drag on the 3 segments, appended to the
      // action for the Thrusters: force_b = rot_b(vel_b * sph - diag(D)),
      // D[b][k] = fix_k |v_bk| v_bk in the segment frame, and jp.diag keeps
      // D's diagonal (D00, D11, D22) for every segment (the reference's
      // broadcast); clipped to [-5, 5]
      const float* q = E.qp + lane * QP_STRIDE;
      q4 rot{0.f, 0.f, 0.f, 0.f};
      v3 vel = mk(0.f, 0.f, 0.f);
      if (lane < 3) {
        rot = q4{q[3], q[4], q[5], q[6]};
        vel = ld3(q + 7);
        v3 lv = rotate(vel, quat_inv(rot));
        float l = lane == 0 ? lv.x : (lane == 1 ? lv.y : lv.z);
        E.red[60 + lane] = P.coef[3 + lane] * fabsf(l) * l;
      }
      esync<L>();
      if (lane < 3 && valid) {
        v3 f = vel * P.coef[2] - mk(E.red[60], E.red[61], E.red[62]);
        f = rotate(f, rot);
        xact[aw + 3 * lane] = clampf(f.x, -5.f, 5.f);
        xact[aw + 3 * lane + 1] = clampf(f.y, -5.f, 5.f);
        xact[aw + 3 * lane + 2] = clampf(f.z, -5.f, 5.f);
      }
      if (valid && lane < aw) xact[lane] = act[lane];
      sact = valid ? xact : nullptr;
      saw = aw + 9;
    } else if (KIND_IS(BX_ENV_GRASP)) {
      // grasp.py:63-77: the [-1, 1] action mapped onto the angle limits and
      // the palm's range; the palm moves 15 % of the way to the last three
      // (at most 2 units) before the physics
      for (int i = lane; i < aw; i += L)
        if (valid) xact[i] = P.act_map[i] + P.act_map[aw + i] * ((act[i] + 1.f) / 2.f);
      esync<L>();
      if (lane == 0 && valid) {
        float* pp = E.qp + (int)P.coef[0] * QP_STRIDE;
        v3 palm = ld3(pp);
        v3 d = mk(xact[aw - 3], xact[aw - 2], xact[aw - 1]) - palm;
        float nrm = norm(d);
        float scl = nrm > 2.f ? 2.f / nrm : 1.f;
        st3(pp, palm + scl * d * .15f);
      }
      sact = valid ? xact : nullptr;
    }
    esync<L>();
    if constexpr (S) {
      v3 ica, iaa;
      pbd_step_single<L, F, M, EK != EK_ANY, true>(c, H, E, lane, valid, sact, saw, X, icv, ica, iaa);
    } else if (H.spring) {
      spring_step<L, F>(c, H, E, lane, valid, sact, saw);
    } else {
      pbd_step<L, F>(c, H, E, lane, valid, sact, saw);
    }
    BX_KSTAMP(11);
    // the Humanoid kernel's actuators drive the joints of their own index
    // (its launch requires fold), so its observation takes the lane's
    // hoisted body, joint and actuator
    // (JB: the lane's hoisted body is its joint side's, not body lane)
    constexpr bool JBK = S && (F & F_JH) != 0 && EK != EK_ANY && (F & F_C16) == 0;
    env_observe<L, EK>(c, H, E, lane, kind, P.obs_flags, P.obs_size, act, aw,
                   valid ? O.obs + e * P.obs_size : nullptr, P.coef, S ? &X.J : nullptr,
                   (S && !JBK) ? &X.B : nullptr, (S && EK == EK_HUM) ? &X.A : nullptr);
    BX_KSTAMP(12);
    // the Ant kernel's contact cost: each body lane's clipped squares, summed
    // across the env's lanes by DPP
    float ccs = 0.f;
    if constexpr (S && EK == EK_ANT && L == 16) {
      const v3 cv = mk(clip1(icv.x), clip1(icv.y), clip1(icv.z));
      ccs = row_sum16(X.own ? cv.x * cv.x + cv.y * cv.y + cv.z * cv.z : 0.f);
    }
    // reward / done / metrics (lane 0 of the env)
    if (lane == 0 && valid) {
      const float dt = H.dt;
      float* m = O.metrics ? O.metrics + e * P.n_metrics : nullptr;
      v3 p1 = ld3(E.qp);
      float reward = 0.f;
      if (KIND_IS(BX_ENV_ANT)) {
        v3 vel = (p1 - pos0) / dt;
        float fwd = vel.x;
        float z = p1.z;
        float healthy = in_range_or_nan(z, P.coef[4], P.coef[5]) ? 1.f : 0.f;
        bool term = P.coef[6] != 0.f;
        float hr = term ? P.coef[3] : P.coef[3] * healthy;
        float ctrl = P.coef[1] * sq;
        float cs = ccs;
        if constexpr (!(S && EK == EK_ANT && L == 16))
          for (int b = 0; b < H.N; b++)
            for (int k = 0; k < 3; k++) {
              float cv = clip1(E.acc[b * ACC_STRIDE + ACC_ICV + k]);
              cs += cv * cv;
            }
        float ccost = P.coef[2] * cs;
        reward = fwd + hr - ctrl - ccost;
        done = term ? 1.f - healthy : 0.f;
        if (m) {
          m[0] = norm(p1); m[1] = fwd; m[2] = -ccost; m[3] = -ctrl; m[4] = fwd;
          m[5] = hr; m[6] = p1.x; m[7] = vel.x; m[8] = p1.y; m[9] = vel.y;
        }
      } else if (KIND_IS(BX_ENV_HALFCHEETAH)) {
        float v0 = (p1.x - pos0.x) / dt;
        float fwd = P.coef[0] * v0;
        float ctrl = P.coef[1] * sq;
        reward = fwd - ctrl;
        if (m) { m[0] = -ctrl; m[1] = fwd; m[2] = p1.x; m[3] = v0; }
      } else if (KIND_IS(BX_ENV_HUMANOID)) {
        v3 com1 = ld3(E.red + 32);
        v3 v = (com1 - com0) / dt;
        float fwd = P.coef[0] * v.x;
        float z = p1.z;
        float healthy = in_range_or_nan(z, P.coef[4], P.coef[5]) ? 1.f : 0.f;
        bool term = P.coef[6] != 0.f;
        float hr = term ? P.coef[3] : P.coef[3] * healthy;
        float ctrl = P.coef[1] * sq;
        reward = fwd + hr - ctrl;
        done = term ? 1.f - healthy : 0.f;
        if (m) {
          m[0] = norm(com1); m[1] = fwd; m[2] = hr; m[3] = fwd; m[4] = -ctrl;
          m[5] = com1.x; m[6] = v.x; m[7] = com1.y; m[8] = v.y;
        }
      } else if (KIND_IS(BX_ENV_HOPPER) || KIND_IS(BX_ENV_WALKER2D)) {
        // hopper.py:204-229 / walker2d.py: healthy z and torso pitch ranges
        float xv = (p1.x - pos0.x) / dt;
        float fwd = P.coef[0] * xv;
        float ay = euler_y(E.qp + 3);
        float z = p1.z;
        float healthy = in_range_or_nan(z, P.coef[3], P.coef[4]) &&
                        in_range_or_nan(ay, P.coef[5], P.coef[6]) ? 1.f : 0.f;
        bool term = P.coef[7] != 0.f;
        float hr = term ? P.coef[2] : P.coef[2] * healthy;
        float ctrl = P.coef[1] * sq;
        reward = fwd + hr - ctrl;
        done = term ? 1.f - healthy : 0.f;
        // sorted: reward_ctrl, reward_forward, reward_healthy, x_position, x_velocity
        if (m) { m[0] = -ctrl; m[1] = fwd; m[2] = hr; m[3] = p1.x; m[4] = xv; }
      } else if (KIND_IS(BX_ENV_INVERTED_PENDULUM)) {
        reward = 1.f;
        done = fabsf(E.ang[0]) > .2f && !is_nan(E.ang[0]) ? 1.f : 0.f;  // |obs[1]| > .2
      } else if (KIND_IS(BX_ENV_INVERTED_DOUBLE_PENDULUM)) {
        // the pole tip (body 2's (0, 0, .3)) in the world
        const float* q2 = E.qp + 2 * QP_STRIDE;
        v3 tip = ld3(q2) + rotate(mk(0.f, 0.f, .3f), q4{q2[3], q2[4], q2[5], q2[6]});
        float x = tip.x, y = tip.z;
        float dist = 0.01f * (x * x) + (y - 2.f) * (y - 2.f);
        float v1 = E.ang[H.D], v2 = E.ang[H.D + 1];
        float velp = 1e-3f * (v1 * v1) + 5e-3f * (v2 * v2);
        reward = 10.f - dist - velp;
        done = y <= 1.f && !is_nan(y) ? 1.f : 0.f;
      } else if (KIND_IS(BX_ENV_ACROBOT)) {
        float a0 = E.ang[0], a1 = E.ang[1], w0 = E.ang[H.D], w1 = E.ang[H.D + 1];
        float dist = a0 * a0 + a1 * a1;
        float velp = 1e-3f * (w0 * w0 + w1 * w1);
        reward = 10.f - dist - velp;
        done = 0.f;
        // sorted: alive_bonus (never updated: stays at its reset 0), dist_penalty, r_tot, vel_penalty
        if (m) { m[0] = 0.f; m[1] = dist; m[2] = reward; m[3] = velp; }
      } else if (KIND_IS(BX_ENV_REACHER) || KIND_IS(BX_ENV_REACHERANGLE)) {
        // reacher.py:188-197 / reacherangle.py:79-95: -|tip - target| (- |a|^2)
        v3 tp, tv;
        arm_tip(E, P.coef, tp, tv);
        float rd = -norm(tp - ld3(E.qp + (int)P.coef[0] * QP_STRIDE));
        if (KIND_IS(BX_ENV_REACHER)) {
          float rc = -sq;
          reward = rd + rc;
          if (m) { m[0] = rc; m[1] = rd; }  // sorted: reward_ctrl, reward_dist
        } else {
          reward = rd;
          if (m) { m[0] = 0.f; m[1] = rd; }  // sorted: rewardCtrl, rewardDist
        }
      } else if (KIND_IS(BX_ENV_SWIMMER)) {
        // swimmer.py:222-241: the segments' centre of mass; done as it came in
        v3 com1;
        humanoid_com(c, H, E.qp, com1, msum);
        v3 v = (com1 - com0) / dt;
        float fwd = P.coef[0] * v.x;
        float ctrl = P.coef[1] * sq;
        reward = fwd - ctrl;
        // sorted: distance_from_origin, forward_reward, reward_ctrl, reward_fwd,
        // x_position, x_velocity, y_position, y_velocity
        if (m) {
          m[0] = norm(p1); m[1] = fwd; m[2] = -ctrl; m[3] = fwd;
          m[4] = com1.x; m[5] = v.x; m[6] = com1.y; m[7] = v.y;
        }
      } else if (KIND_IS(BX_ENV_UR5E) || KIND_IS(BX_ENV_FETCH)) {
        // ur5e.py:82-101 / fetch.py:58-99 (done as it came in); a hit target
        // moves to a fresh spot drawn from the env's stream (after the obs)
        const int ti = (int)P.coef[0], gi = (int)P.coef[1];
        v3 t1 = ld3(E.qp + ti * QP_STRIDE);
        v3 delta = t1 - ld3(E.red + 36);  // torso before the step
        v3 rel = ld3(E.qp + gi * QP_STRIDE) - t1;
        float dist = norm(rel);
        v3 dir = rel / (1e-6f + dist);
        float moving = .1f * dot(delta, dir);
        float hit = dist < P.coef[2] ? 1.f : 0.f;
        const float* tq = E.qp + ti * QP_STRIDE;
        const q4 tr{tq[3], tq[4], tq[5], tq[6]};
        if (KIND_IS(BX_ENV_UR5E)) {
          reward = moving + hit;
          if (m) { m[0] = hit; m[1] = moving; m[2] = hit; }  // sorted: hits, movingToTarget, weightedHits
        } else {
          v3 up = rotate(mk(0.f, 0.f, 1.f), tr);
          float is_up = .1f * dt * dot(up, mk(0.f, 0.f, 1.f));
          float height = .1f * dt * E.qp[2];
          float facing = dot(dir, rotate(mk(1.f, 0.f, 0.f), tr));
          float whit = hit * facing;
          reward = height + moving + is_up + whit;
          // sorted: hits, movingToTarget, torsoHeight, torsoIsUp, weightedHits
          if (m) { m[0] = hit; m[1] = moving; m[2] = height; m[3] = is_up; m[4] = whit; }
        }
        // one draw per env step (action repeats included), as the reference
        // splits its key once per step
        const uint32_t key = rng_c + (uint32_t)rep;
        if (rep == reps - 1) O.rng[e] = key + 1u;
        if (hit != 0.f) {
          float u0 = uniform_at(key, 0, 0.f, 1.f), u1 = uniform_at(key, 1, 0.f, 1.f);
          float rr = P.coef[2] + P.coef[3] * u0;
          float an = 3.14159265358979323846f * 2.f * u1;
          float* g = E.qp + gi * QP_STRIDE;
          g[0] = rr * cosf(an);
          g[1] = rr * sinf(an);
          g[2] = P.coef[4];
        }
      } else if (KIND_IS(BX_ENV_GRASP)) {
        // grasp.py:80-126 (done as it came in); a hit target moves to a
        // fresh spot from the env's stream (after the obs)
        const int oi = (int)P.coef[1], gi = (int)P.coef[2], hi = (int)P.coef[3];
        v3 op = ld3(E.qp + oi * QP_STRIDE), hp = ld3(E.qp + (int)P.coef[0] * QP_STRIDE);
        v3 hv = ld3(E.qp + hi * QP_STRIDE + 7);
        v3 rel = op - hp;
        float od = norm(rel);
        float planar = norm(mul(rel, mk(1.f, 1.f, 0.f)));
        v3 odir = rel / (1e-6f + od);
        float mto = .1f * dt * dot(hv, odir);
        float close = .1f * dt * 1.f / (1.f + planar);
        v3 trel = ld3(E.qp + gi * QP_STRIDE) - op;
        float td = norm(trel);
        v3 tdir = trel / (1e-6f + td);
        float mtt = 1.5f * dt * dot(ld3(E.qp + oi * QP_STRIDE + 7), tdir);
        float touch = 0.f;
        const int tb[4] = {3, 9, 12, 15};
        for (int k = 0; k < 4; k++) {
          const float* cv = E.acc + tb[k] * ACC_STRIDE + ACC_ICV;
          touch += cv[0] * cv[0] + cv[1] * cv[1] + cv[2] * cv[2] > 0.00001f ? 1.f : 0.f;
        }
        touch = 0.2f * dt * touch;
        float hit = td < P.coef[4] ? 1.f : 0.f;
        reward = mto + close + touch + 5.f * hit + mtt;
        // sorted: closeToObject, hits, movingObjectToTarget, movingToObject, touchingObject
        if (m) { m[0] = close; m[1] = hit; m[2] = mtt; m[3] = mto; m[4] = touch; }
        const uint32_t key = rng_c + (uint32_t)rep;
        if (rep == reps - 1) O.rng[e] = key + 1u;
        if (hit != 0.f) {
          float u0 = uniform_at(key, 0, 0.f, 1.f), u1 = uniform_at(key, 1, 0.f, 1.f);
          float u2 = uniform_at(key, 2, 0.f, 1.f);
          float rr = P.coef[4] + P.coef[5] * u0;
          float an = 3.14159265358979323846f * 2.f * u1;
          float* g = E.qp + gi * QP_STRIDE;
          g[0] = rr * cosf(an);
          g[1] = rr * sinf(an);
          g[2] = P.coef[6] * u2;
        }
      } else if (KIND_IS(BX_ENV_PUSHER)) {
        // pusher.py:212-231; done as it came in
        float rc = -sq;
        reward = dist0 + 0.1f * rc + 0.5f * near0;
        if (m) { m[0] = rc; m[1] = dist0; m[2] = near0; }  // sorted: ctrl, dist, near
      } else if (KIND_IS(BX_ENV_HUMANOID_STANDUP)) {
        // humanoid_standup.py:232-247: uph = z / dt, reward = uph + 1 - 0.01 sum(a^2);
        // done is left as it came in
        float uph = (p1.z - 0.f) / dt;
        float ctrl = P.coef[1] * sq;
        reward = uph + 1.f - ctrl;
        if (m) { m[0] = uph; m[1] = -ctrl; }
      }
      reward_sum = rep == 0 ? reward : reward_sum + reward;
      E.red[0] = done;
    }
    esync<L>();
  }
  BX_KSTAMP(13);
  done = E.red[0];
  float trunc = 0.f;
  bool reset_now = false;
  if (P.episode_length > 0) {
    steps = steps + (float)reps;
    float ep = (float)P.episode_length;
    float d_inner = done;
    done = steps >= ep ? 1.f : d_inner;
    trunc = steps >= ep ? 1.f - d_inner : 0.f;
  }
  if (P.auto_reset) reset_now = done != 0.f;
  if (valid) {
    if (lane == 0) {
      O.reward[e] = reward_sum;
      O.done[e] = done;
      if (O.steps) O.steps[e] = steps;
      if (O.truncation) O.truncation[e] = trunc;
    }
    if (reset_now) {
      for (int b = lane; b < H.N; b += L) {
        float tmp[13];
        load_qp_global(P.first_qp, e, b, tmp);
        store_out_qp(b, tmp);
        // the next step starts from the reset state
        if (t + 1 < nst) {
          float* s = E.qp + b * QP_STRIDE;
#pragma unroll
          for (int k = 0; k < 13; k++) s[k] = tmp[k];
        }
      }
      for (int i = lane; i < P.obs_size; i += L) O.obs[e * P.obs_size + i] = P.first_obs[e * P.obs_size + i];
    } else {
      for (int b = lane; b < H.N; b += L) store_out_qp(b, E.qp + b * QP_STRIDE);
    }
  }
  // the next step's input scalars: this step's outputs
  done_in = done;
  steps_in = steps;
  rng_c += (uint32_t)reps;
  esync<L>();
  }  // steps
  BX_KSTAMP(14);
}



template <int L, int MODE, int F, int M, int EK = EK_ANY>
__global__ void __launch_bounds__(L > 64 ? L : 64) BX_STEP_ATTR env_step_kernel(EnvArgs A) {
  env_step_body<L, MODE, F, M, EK>(A);
}
// one step on the packed layout (bx_env_step_packed: Env.step's host path)
// through the PK body, under its own name (the benchmarked envs' kernels)
template <int L, int MODE, int F, int M, int EK = EK_ANY>
__global__ void __launch_bounds__(L > 64 ? L : 64) BX_STEP_ATTR env_step_packed_kernel(EnvArgs A) {
  env_step_body<L, MODE, F, M, EK, true, true>(A);
}
// the Ant step kernel held to 256 registers (2 waves per SIMD) for batches
// past one wave per SIMD: at 4,096 envs the unbounded kernel's single wave
// per SIMD is 7 % faster (29.8 vs 32.0 us), but at 32,768 envs (8 waves per
// SIMD) it runs 8 residency rounds against this one's 4 (152 vs 219 M
// env-steps/s, tools/ab_ant_waves.sh)
template <int L, int MODE, int F, int M, int EK = EK_ANY>
__global__ void __launch_bounds__(L > 64 ? L : 64) __attribute__((amdgpu_waves_per_eu(2)))
env_step_wide_kernel(EnvArgs A) {
  env_step_body<L, MODE, F, M, EK>(A);
}
template <int L, int MODE, int F, int M, int EK = EK_ANY>
__global__ void __launch_bounds__(L > 64 ? L : 64) __attribute__((amdgpu_waves_per_eu(2)))
env_rollout_wide_kernel(EnvArgs A) {
  env_step_body<L, MODE, F, M, EK, true>(A);
}
// the same body under its own name for multi-step launches of the
// benchmarked envs' kernels (bx_env_rollout_packed), so a profile tells
// K-step launches from single steps
template <int L, int MODE, int F, int M, int EK = EK_ANY>
__global__ void __launch_bounds__(L > 64 ? L : 64) BX_STEP_ATTR env_rollout_kernel(EnvArgs A) {
  env_step_body<L, MODE, F, M, EK, true>(A);
}

// System.info contact part + optional Env._get_obs of the same state (reset)
template <int L>
__global__ void __launch_bounds__(L > 64 ? L : 64) info_obs_kernel(InfoArgs A) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  Cst c{A.blob};
  BlobHdr H = *reinterpret_cast<const BlobHdr*>(A.blob);
  const int lane = threadIdx.x % L;
  const int le = threadIdx.x / L;
  const int64_t e = (int64_t)blockIdx.x * (blockDim.x / L) + le;
  const bool valid = e < A.n_envs;
  Env E = carve(smem + le * H.env_words, H);
  if (valid) {
    for (int b = lane; b < H.N; b += L) load_qp_global(A.q, e, b, E.qp + b * QP_STRIDE);
  } else {
    for (int b = lane; b < H.N; b += L) {
      float* s = E.qp + b * QP_STRIDE;
      for (int k = 0; k < 13; k++) s[k] = k == 3 ? 1.f : 0.f;
    }
  }
  esync<L>();
  if (A.angle) {  // Joint.angle_vel only
    joint_angles<L>(c, H, E, lane);
    esync<L>();
    if (valid)
      for (int i = lane; i < H.D; i += L) {
        A.angle[e * H.D + i] = E.ang[i];
        A.angvel[e * H.D + i] = E.ang[H.D + i];
      }
    return;
  }
  pbd_info<L>(c, H, E, lane);
  if (valid) {
    for (int b = lane; b < H.N; b += L) {
      const float* acc = E.acc + b * ACC_STRIDE;
      const bx_info& I = A.info;
      if (I.contact_vel.ptr) {
        float* p = I.contact_vel.ptr + e * I.contact_vel.env_stride + b * I.contact_vel.body_stride;
        p[0] = acc[ACC_ICV]; p[1] = acc[ACC_ICV + 1]; p[2] = acc[ACC_ICV + 2];
      }
      if (I.contact_ang.ptr) {
        float* p = I.contact_ang.ptr + e * I.contact_ang.env_stride + b * I.contact_ang.body_stride;
        p[0] = acc[ACC_ICA]; p[1] = acc[ACC_ICA + 1]; p[2] = acc[ACC_ICA + 2];
      }
    }
  }
  if (A.obs) {
    const float* act = valid && A.act ? A.act + e * A.act_stride : nullptr;
    env_observe<L>(c, H, E, lane, A.kind, A.obs_flags, A.obs_size, act, (int)A.act_width,
                   valid ? A.obs + e * A.obs_size : nullptr, A.coef);
  }
  // reset: reward, done, steps, truncation and metrics start at zero
  // (ant.py:205-219, wrappers.py:94-97)
  if (valid) {
    if (lane == 0) {
      if (A.zero_reward) A.zero_reward[e] = 0.f;
      if (A.zero_done) A.zero_done[e] = 0.f;
      if (A.zero_steps) A.zero_steps[e] = 0.f;
      if (A.zero_trunc) A.zero_trunc[e] = 0.f;
    }
    if (A.zero_metrics)
      for (int i = lane; i < A.n_metrics; i += L) A.zero_metrics[e * A.n_metrics + i] = 0.f;
  }
}


// System.default_qp (system.py:112-242): one thread per env (reset path)


#if !defined(BX_TU_FAST)  // reset / RNG kernels: the generic translation unit
__global__ void __launch_bounds__(64) default_qp_kernel(ResetArgs A) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  Cst c{A.blob};
  BlobHdr H = *reinterpret_cast<const BlobHdr*>(A.blob);
  const int64_t e = (int64_t)blockIdx.x * 64 + threadIdx.x;
  if (e >= A.n_envs) return;
  float* q = smem + threadIdx.x * H.N * 13;  // per-thread scratch: N x 13
  const int N = H.N, D = H.num_joint_dof;
  for (int b = 0; b < N; b++)
    for (int k = 0; k < 13; k++) q[b * 13 + k] = c.f(H.o_base + b * 13 + k);
  const float* ja = A.gen ? nullptr : A.angle + e * D;
  const float* jv = A.gen ? nullptr : A.vel + e * D;
  // Env.reset draws (gen = 1), keyed by the global env id g (W draws per
  // env: (seed, g * W + k)) or by the env's own key (seeds[e], k):
  //   default (ant.py:200-203 ...): qpos = default + U[-s, s) at k = dof,
  //     qvel = U[-s, s) at k = D + dof (W = 2D)
  //   REACHER, REACHERANGLE (reacher.py:157-160): qpos noise U[-.1, .1),
  //     qvel U[-.005, .005), then the target's two draws at 2D, 2D + 1
  //   PUSHER (pusher.py:178-195): default angles, qvel U[-.005, .005) on the
  //     first D - 4 dofs (k = dof), the object's two draws at D - 4, D - 3
  //   UR5E, FETCH (ur5e.py:41-46): default pose at rest, the target's two
  //     draws at 0, 1;  GRASP (grasp.py:54-70): default pose at rest
  const int kind = A.gen ? A.kind : 0;
  int W = 2 * D;
  float as = A.scale, vs = A.scale;
  int nvel = D;
  if (kind == BX_ENV_REACHER || kind == BX_ENV_REACHERANGLE) {
    W = 2 * D + 2; as = .1f; vs = .005f;
  } else if (kind == BX_ENV_PUSHER) {
    W = D - 4 + 2; as = 0.f; vs = .005f; nvel = D - 4;
  } else if (kind == BX_ENV_UR5E || kind == BX_ENV_FETCH) {
    W = 2; as = 0.f; vs = 0.f; nvel = 0;
  } else if (kind == BX_ENV_GRASP) {
    W = 0; as = 0.f; vs = 0.f; nvel = 0;
  }
  const int voff = kind == BX_ENV_PUSHER ? 0 : D;  // pusher's qvel draws come first
  const uint64_t seed = A.seeds ? A.seeds[e] : A.seed;
  const uint64_t g0 = A.seeds ? 0ull : (uint64_t)(A.env_offset + e) * (uint64_t)W;
  for (int f = 0; f < H.n_fk; f++) {
    int o = H.o_fk + f * FK_STRIDE;
    float a3[3], v3_[3];
    for (int l = 0; l < 3; l++) {
      int ix = c.i(o + FK_IDX + l);
      if (A.gen) {
        a3[l] = ix < 0 ? 0.f
                : c.f(H.o_dangle + ix) + (as > 0.f ? uniform_at(seed, g0 + ix, -as, as) : 0.f);
        v3_[l] = ix >= 0 && ix < nvel ? uniform_at(seed, g0 + voff + ix, -vs, vs) : 0.f;
      } else {
        a3[l] = ix >= 0 ? ja[ix] : 0.f;
        v3_[l] = ix >= 0 ? jv[ix] : 0.f;
      }
    }
    q4 jr{c.f(o + FK_ROT), c.f(o + FK_ROT + 1), c.f(o + FK_ROT + 2), c.f(o + FK_ROT + 3)};
    q4 rot{c.f(o + FK_REF), c.f(o + FK_REF + 1), c.f(o + FK_REF + 2), c.f(o + FK_REF + 3)};
    v3 axes[3] = {rotate(mk(1.f, 0.f, 0.f), jr), rotate(mk(0.f, 1.f, 0.f), jr),
                  rotate(mk(0.f, 0.f, 1.f), jr)};
    v3 lang = axes[0] * v3_[0] + axes[1] * v3_[1] + axes[2] * v3_[2];
    for (int l = 0; l < 3; l++) {
      v3 ax = rotate(axes[l], rot);
      rot = quat_mul(quat_rot_axis(ax, a3[l]), rot);
    }
    int bp = c.i(o + FK_BP), bc = c.i(o + FK_BC);
    float* sp = q + bp * 13;
    float* sc = q + bc * 13;
    q4 prot = ld4(sp + 3);
    q4 wr = quat_mul(prot, rot);
    v3 lp = c.f3(o + FK_OFFP) - rotate(c.f3(o + FK_OFFC), rot);
    v3 wp = ld3(sp) + rotate(lp, prot);
    v3 wa = rotate(lang, prot);
    st3(sc, wp);
    st4(sc + 3, wr);
    st3(sc + 10, wa);
  }
  // bodies.min_z per root group, then lift (system.py:213-240)
  for (int g = 0; g < H.n_root_groups; g++) {
    float zmin = 3.4028235e38f;
    for (int b = 0; b < N; b++) {
      if (c.i(H.o_rgroup + b) != g) continue;
      float bz = 3.4028235e38f;
      for (int p = c.i(H.o_zoff + b), pe = c.i(H.o_zoff + b + 1); p < pe; p++) {
        int o = H.o_zpt + p * 4;
        v3 w = rotate(c.f3(o), ld4(q + b * 13 + 3));
        float z = q[b * 13 + 2] + w.z - c.f(o + 3);
        bz = fminf(bz, z);
      }
      if (c.i(H.o_zero + b)) bz = fminf(bz, 0.f);
      zmin = fminf(zmin, bz);
    }
    for (int b = 0; b < N; b++) {
      if (c.i(H.o_rgroup + b) != g) continue;
      q[b * 13 + 0] = q[b * 13 + 0] - zmin * 0.f;
      q[b * 13 + 1] = q[b * 13 + 1] - zmin * 0.f;
      q[b * 13 + 2] = q[b * 13 + 2] - zmin * 1.f;
    }
  }
  // the bodies the env's reset places after default_qp (index_update of
  // qp.pos, so after the lift): the reachers' target (reacher.py:212-221,
  // reacherangle.py:102-113: radius .2 u, sqrt(u) for ReacherAngle), the
  // pusher's object in its .17 disc, goal and table (pusher.py:181-201), the
  // target envs' target on their ring (ur5e.py:117-125, fetch.py:124-134)
  const float twopi = 3.14159265358979323846f * 2.f;
  if (kind == BX_ENV_REACHER || kind == BX_ENV_REACHERANGLE) {
    const float u0 = uniform_at(seed, g0 + 2 * D, 0.f, 1.f);
    const float u1 = uniform_at(seed, g0 + 2 * D + 1, 0.f, 1.f);
    const float dist = .2f * (kind == BX_ENV_REACHERANGLE ? sqrtf(u0) : u0);
    const float an = twopi * u1;
    float* t = q + (int)A.coef[0] * 13;
    t[0] = dist * cosf(an);
    t[1] = dist * sinf(an);
    t[2] = .01f;
  } else if (kind == BX_ENV_PUSHER) {
    float x = uniform_at(seed, g0 + D - 4, -.3f, 0.f);
    float y = uniform_at(seed, g0 + D - 3, -.2f, .2f);
    const float nrm = sqrtf(x * x + y * y);
    const float sc = nrm > .17f ? .17f / nrm : 1.f;
    float* ob = q + (int)A.coef[1] * 13;
    ob[0] = sc * x;
    ob[1] = sc * y;
    ob[2] = .05f;
    float* gl = q + (int)A.coef[2] * 13;
    gl[0] = .45f; gl[1] = .05f; gl[2] = .05f;
    float* tb = q + (int)A.coef[3] * 13;
    tb[0] = 0.f; tb[1] = 0.f; tb[2] = 0.f;
  } else if (kind == BX_ENV_UR5E || kind == BX_ENV_FETCH) {
    const float u0 = uniform_at(seed, g0, 0.f, 1.f), u1 = uniform_at(seed, g0 + 1, 0.f, 1.f);
    const float rr = A.coef[2] + A.coef[3] * u0;
    const float an = twopi * u1;
    float* t = q + (int)A.coef[1] * 13;
    t[0] = rr * cosf(an);
    t[1] = rr * sinf(an);
    t[2] = A.coef[4];
  }
  // the target envs' per-env stream (info['rng']): a hash of (seed, global
  // env id), or of the env's own key
  if (A.rng_out && (kind == BX_ENV_UR5E || kind == BX_ENV_FETCH || kind == BX_ENV_GRASP)) {
    const uint64_t id = A.seeds ? 0ull : (uint64_t)(A.env_offset + e);
    int64_t z = (int64_t)(id * 0x9E3779B97F4A7C15ull + (seed & 0x7FFFFFFFFFFFFFFFull));
    z = (int64_t)((uint64_t)(z ^ (z >> 31)) * 0x94D049BB133111EBull);
    A.rng_out[e] = (uint32_t)(z ^ (z >> 29));
  }
  for (int b = 0; b < N; b++) store_qp_global(A.out, e, b, q + b * 13);
}

// counter-based uniform fill: splitmix64 of (seed, index) -> [lo, hi)
__global__ void uniform_kernel(float* out, int64_t n, uint64_t seed, uint64_t offset, float lo,
                               float hi) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  out[i] = uniform_at(seed, (uint64_t)i + offset, lo, hi);
}

// the same fill over n_slabs slabs of slab_n elements with their own offsets,
// advanced by a device-resident epoch counter: out[s * slab_n + j] =
// U(seed, offset + epoch * epoch_stride + s * slab_stride + j). A
// graph-captured rollout draws the action slabs of all its K steps in one
// launch and still draws fresh slabs per replay (the counter is bumped inside
// the graph); epoch null reads as 0
__global__ void uniform_slabs_kernel(float* out, int64_t slab_n, int64_t n, uint64_t seed,
                                     uint64_t offset, uint64_t slab_stride,
                                     const int64_t* __restrict__ epoch, uint64_t epoch_stride,
                                     float lo, float hi) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint64_t e = epoch ? (uint64_t)epoch[0] : 0ull;
  const int64_t sl = i / slab_n, j = i - sl * slab_n;
  out[i] = uniform_at(seed, offset + e * epoch_stride + (uint64_t)sl * slab_stride + (uint64_t)j,
                      lo, hi);
}

#endif

}  // namespace bx

// ---------------------------------------------------------------------------
// launch helpers (host)
// ---------------------------------------------------------------------------
namespace bx {

// compute units of the current device (the launch runs under the system's
// device scope), cached per device
static int cu_count() {
  static int cached[64] = {0};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
  if (!cached[dev]) {
    int n = 0;
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
    cached[dev] = n;
  }
  return cached[dev];
}

template <typename Args>
static void launch_one(void (*k)(Args), dim3 grid, int tpb, size_t lds, hipStream_t s, const Args& a) {
  // tpb threads per workgroup (a multiple of L, <= 64): 64 / L envs share a
  // wavefront by default; 32 halves that (twice the waves for one batch)
  if (lds > 65536) (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  hipLaunchKernelGGL(k, grid, dim3(tpb), lds, s, a);
}

// instantiated variants: (lanes, mode, features, gather width). This file is
// compiled twice (Makefile): BX_TU_FAST holds the register-hoisted SINGLE-mode
// kernels; BX_TU_GENERIC holds the item-loop kernels (large scenes,
// legacy_spring, the extended contact functions) and the reset / info
// kernels. Both are built with fast reciprocal division by default
// (GENERIC_PRECISE=1: IEEE division in the second). Single mode at 16 lanes is
// specialised per feature set and gather width.
#define BX_SINGLE16(KERNEL, ARGS, M)                                                \
  switch (feat) {                                                                   \
    case 0: launch_one<ARGS>(KERNEL<16, 1, 0, M>, grid, tpb, lds, s, a); break;     \
    case F_SPH: launch_one<ARGS>(KERNEL<16, 1, F_SPH, M>, grid, tpb, lds, s, a); break; \
    case F_G1: launch_one<ARGS>(KERNEL<16, 1, F_G1, M>, grid, tpb, lds, s, a); break; \
    case F_SPH | F_G1: launch_one<ARGS>(KERNEL<16, 1, F_SPH | F_G1, M>, grid, tpb, lds, s, a); break; \
    case F_CC | F_TW: launch_one<ARGS>(KERNEL<16, 1, F_CC | F_TW, M>, grid, tpb, lds, s, a); break; \
    case F_CC | F_TW | F_G1: launch_one<ARGS>(KERNEL<16, 1, F_CC | F_TW, M>, grid, tpb, lds, s, a); break; \
    case F_G1 | F_JH: launch_one<ARGS>(KERNEL<16, 1, F_G1 | F_JH, M>, grid, tpb, lds, s, a); break; \
    case F_JH: launch_one<ARGS>(KERNEL<16, 1, F_JH, M>, grid, tpb, lds, s, a); break; \
    case F_CC | F_TW | F_JH: \
    case F_CC | F_TW | F_G1 | F_JH: launch_one<ARGS>(KERNEL<16, 1, F_CC | F_TW | F_JH, M>, grid, tpb, lds, s, a); break; \
    default: launch_one<ARGS>(KERNEL<16, 1, F_ALL, M>, grid, tpb, lds, s, a); break; \
  }
// F_R2 systems (17-32 rows at 16 lanes): HalfCheetah (capsule-capsule,
// two-way, joint halves), Fetch (box corners, one group), HumanoidStandup
// (spherical, one group), else every feature
#define BX_SINGLE16_R2(KERNEL, ARGS, M)                                             \
  if (feat & F_C16) {                                                               \
    if ((feat & ~(F_R2 | F_C16 | F_G1 | F_R2G)) == (F_CC | F_TW | F_JH) && (feat & F_R2G)) \
      launch_one<ARGS>(KERNEL<16, 1, F_CC | F_TW | F_JH | F_R2 | F_C16 | F_R2G, M>, grid, tpb, lds, s, a); \
    else if ((feat & ~(F_R2 | F_C16 | F_G1 | F_R2G)) == (F_CC | F_TW | F_JH))      \
      launch_one<ARGS>(KERNEL<16, 1, F_CC | F_TW | F_JH | F_R2 | F_C16, M>, grid, tpb, lds, s, a); \
    else                                                                            \
      launch_one<ARGS>(KERNEL<16, 1, F_ALL | F_R2 | F_C16, M>, grid, tpb, lds, s, a); \
  } else                                                                            \
  switch (feat & ~F_R2) {                                                           \
    case F_CC | F_TW | F_JH | F_R2G:                                                \
    case F_CC | F_TW | F_G1 | F_JH | F_R2G: launch_one<ARGS>(KERNEL<16, 1, F_CC | F_TW | F_JH | F_R2 | F_R2G, M>, grid, tpb, lds, s, a); break; \
    case F_CC | F_TW | F_JH:                                                        \
    case F_CC | F_TW | F_G1 | F_JH: launch_one<ARGS>(KERNEL<16, 1, F_CC | F_TW | F_JH | F_R2, M>, grid, tpb, lds, s, a); break; \
    case F_G1: launch_one<ARGS>(KERNEL<16, 1, F_G1 | F_R2, M>, grid, tpb, lds, s, a); break; \
    case F_SPH | F_G1: launch_one<ARGS>(KERNEL<16, 1, F_SPH | F_G1 | F_R2, M>, grid, tpb, lds, s, a); break; \
    default: launch_one<ARGS>(KERNEL<16, 1, F_ALL | F_R2, M>, grid, tpb, lds, s, a); break; \
  }
#define BX_DISPATCH_SINGLE(KERNEL, ARGS)                                            \
  if (L == 16 && (feat & F_R2)) {                                                   \
    if (gw <= 4) { BX_SINGLE16_R2(KERNEL, ARGS, 4) } else { BX_SINGLE16_R2(KERNEL, ARGS, 8) } \
  } else if (L == 16 && (feat & F_C16)) {                                           \
    if (gw <= 4) launch_one<ARGS>(KERNEL<16, 1, F_ALL | F_C16, 4>, grid, tpb, lds, s, a); \
    else launch_one<ARGS>(KERNEL<16, 1, F_ALL | F_C16, 8>, grid, tpb, lds, s, a);     \
  } else if (L == 16) {                                                             \
    if (gw <= 4) { BX_SINGLE16(KERNEL, ARGS, 4) } else { BX_SINGLE16(KERNEL, ARGS, 8) } \
  } else if (L == 32) {                                                             \
    launch_one<ARGS>(KERNEL<32, 1, F_ALL, 8>, grid, tpb, lds, s, a);                \
  } else {                                                                          \
    launch_one<ARGS>(KERNEL<64, 1, F_ALL, 8>, grid, tpb, lds, s, a);                \
  }
// item-loop kernels: a lean instantiation (revolute joints, torque
// actuators, capsule-plane / capsule-capsule rows one- or two-way, no forces:
// Ant Mountain, the culled scenes) where the system allows, else every feature
#define F_LEAN (F_CC | F_TW)
#define BX_DISPATCH_GENERIC(KERNEL, ARGS)                                           \
  const bool lean = (feat & (F_SPH | F_ANGLE | F_FORCE | F_X)) == 0;                \
  switch (L * 8 + mode * 2 + (lean ? 1 : 0)) {                                      \
    case 16 * 8 + 0: case 16 * 8 + 1: launch_one<ARGS>(KERNEL<16, 0, F_GEN, 8>, grid, tpb, lds, s, a); break; \
    case 16 * 8 + 4: case 16 * 8 + 5: launch_one<ARGS>(KERNEL<16, 2, F_GEN, 8>, grid, tpb, lds, s, a); break; \
    case 32 * 8 + 0: case 32 * 8 + 1: launch_one<ARGS>(KERNEL<32, 0, F_GEN, 8>, grid, tpb, lds, s, a); break; \
    case 32 * 8 + 4: case 32 * 8 + 5: launch_one<ARGS>(KERNEL<32, 2, F_GEN, 8>, grid, tpb, lds, s, a); break; \
    case 64 * 8 + 0: launch_one<ARGS>(KERNEL<64, 0, F_GEN, 8>, grid, tpb, lds, s, a); break; \
    case 64 * 8 + 1: launch_one<ARGS>(KERNEL<64, 0, F_LEAN, 8>, grid, tpb, lds, s, a); break; \
    case 64 * 8 + 4: case 64 * 8 + 5: launch_one<ARGS>(KERNEL<64, 2, F_GEN, 8>, grid, tpb, lds, s, a); break; \
    case 128 * 8 + 0: launch_one<ARGS>(KERNEL<128, 0, F_GEN, 8>, grid, tpb, lds, s, a); break; \
    case 128 * 8 + 1: launch_one<ARGS>(KERNEL<128, 0, F_LEAN, 8>, grid, tpb, lds, s, a); break; \
    case 256 * 8 + 0: launch_one<ARGS>(KERNEL<256, 0, F_GEN, 8>, grid, tpb, lds, s, a); break; \
    case 256 * 8 + 1: launch_one<ARGS>(KERNEL<256, 0, F_LEAN, 8>, grid, tpb, lds, s, a); break; \
    default: return hipErrorInvalidValue;                                           \
  }

#if defined(BX_TU_FAST)
hipError_t launch_system_step_single(int L, int feat, int gw, int tpb, int64_t n_envs, size_t lds,
                                     hipStream_t s, const StepArgs& a) {
  const int epb = tpb / L;
  dim3 grid((unsigned)((n_envs + epb - 1) / epb));
  BX_DISPATCH_SINGLE(system_step_kernel, StepArgs)
  return hipGetLastError();
}
// single_kernel_feat: BX_DISPATCH_SINGLE run over a host-side probe that
// records the instantiation's F instead of launching it (the same decision)
struct ProbeArgs {
  int* out;
};
template <int PL, int PMODE, int PF, int PM>
void probe_kernel(ProbeArgs a) { *a.out = PF; }
template <>
void launch_one<ProbeArgs>(void (*k)(ProbeArgs), dim3, int, size_t, hipStream_t, const ProbeArgs& a) {
  k(a);
}
int single_kernel_feat(int L, int feat, int gw) {
  int f = -1;
  const ProbeArgs a{&f};
  const dim3 grid(1);
  const int tpb = 64;
  const size_t lds = 0;
  hipStream_t s = nullptr;
  BX_DISPATCH_SINGLE(probe_kernel, ProbeArgs)
  return f;
}
hipError_t launch_env_step_single(int L, int feat, int gw, int tpb, int64_t n_envs, size_t lds,
                                  hipStream_t s, const EnvArgs& a, int fold) {
  const int epb = tpb / L;
  dim3 grid((unsigned)((n_envs + epb - 1) / epb));
  // the benchmarked envs get kernels holding only their own env program
  const int k = a.P.kind;
  // (their kernels fold each joint's damping into its actuator's slot: fold
  // bit 0 = every joint j has torque actuator j; the joint-halves kernels
  // also give each side lane its body's copy: bit 1 = the system allows it)
  const bool jb = (fold & 2) != 0;
  if (fold && jb && L == 16 && gw <= 4 && k == BX_ENV_ANT && feat == (F_G1 | F_JH)) {
    // past one wave per SIMD: the register-capped kernels
    const bool wide = (int64_t)grid.x * (tpb / 64 > 0 ? tpb / 64 : 1) > 4 * (int64_t)cu_count();
    // (a packed single step at a wide batch takes the wide rollout kernel)
    if ((a.n_steps > 1 || a.packed) && wide)
      launch_one<EnvArgs>(env_rollout_wide_kernel<16, 1, F_G1 | F_JH, 4, EK_ANT>, grid, tpb, lds, s, a);
    else if (a.n_steps > 1)
      launch_one<EnvArgs>(env_rollout_kernel<16, 1, F_G1 | F_JH, 4, EK_ANT>, grid, tpb, lds, s, a);
    else if (wide)
      launch_one<EnvArgs>(env_step_wide_kernel<16, 1, F_G1 | F_JH, 4, EK_ANT>, grid, tpb, lds, s, a);
    else if (a.packed)
      launch_one<EnvArgs>(env_step_packed_kernel<16, 1, F_G1 | F_JH, 4, EK_ANT>, grid, tpb, lds, s, a);
    else
      launch_one<EnvArgs>(env_step_kernel<16, 1, F_G1 | F_JH, 4, EK_ANT>, grid, tpb, lds, s, a);
    return hipGetLastError();
  }
  if (fold && L == 16 && gw <= 4 && (k == BX_ENV_HUMANOID || k == BX_ENV_HUMANOID_STANDUP) &&
      feat == (F_SPH | F_G1)) {
    if (a.n_steps > 1)
      launch_one<EnvArgs>(env_rollout_kernel<16, 1, F_SPH | F_G1, 4, EK_HUM>, grid, tpb, lds, s, a);
    else if (a.packed)
      launch_one<EnvArgs>(env_step_packed_kernel<16, 1, F_SPH | F_G1, 4, EK_HUM>, grid, tpb, lds, s, a);
    else
      launch_one<EnvArgs>(env_step_kernel<16, 1, F_SPH | F_G1, 4, EK_HUM>, grid, tpb, lds, s, a);
    return hipGetLastError();
  }
  // HalfCheetah: 16 one-way ground rows in slot 1, the feet's capsule-capsule
  // row in slot 2 (F_R2 | F_R2G), joint halves
  constexpr int F_CHEETAH = F_CC | F_TW | F_JH | F_R2 | F_R2G;
  if (fold && jb && L == 16 && gw <= 4 && k == BX_ENV_HALFCHEETAH && (feat & ~F_G1) == F_CHEETAH) {
    if (a.n_steps > 1)
      launch_one<EnvArgs>(env_rollout_kernel<16, 1, F_CHEETAH, 4, EK_CHEETAH>, grid, tpb, lds, s, a);
    else if (a.packed)
      launch_one<EnvArgs>(env_step_packed_kernel<16, 1, F_CHEETAH, 4, EK_CHEETAH>, grid, tpb, lds, s, a);
    else
      launch_one<EnvArgs>(env_step_kernel<16, 1, F_CHEETAH, 4, EK_CHEETAH>, grid, tpb, lds, s, a);
    return hipGetLastError();
  }
  // Pusher: 16 one-way plane rows in slot 1, 7 two-way capsule-capsule rows
  // as contact halves in slot 2, 16-entry contact lists, joint halves, the
  // damping folded (no body copies: F_C16)
  constexpr int F_PUSHER = F_CC | F_TW | F_JH | F_R2 | F_C16 | F_R2G;
  if (fold && L == 16 && k == BX_ENV_PUSHER && (feat & ~F_G1) == F_PUSHER) {
#define BX_PUSHER_LAUNCH(MW)                                                                        \
    if (a.n_steps > 1)                                                                              \
      launch_one<EnvArgs>(env_rollout_kernel<16, 1, F_PUSHER, MW, EK_PUSHER>, grid, tpb, lds, s, a); \
    else if (a.packed)                                                                              \
      launch_one<EnvArgs>(env_step_packed_kernel<16, 1, F_PUSHER, MW, EK_PUSHER>, grid, tpb, lds, s, a); \
    else                                                                                            \
      launch_one<EnvArgs>(env_step_kernel<16, 1, F_PUSHER, MW, EK_PUSHER>, grid, tpb, lds, s, a);
    if (gw <= 4) { BX_PUSHER_LAUNCH(4) } else { BX_PUSHER_LAUNCH(8) }
#undef BX_PUSHER_LAUNCH
    return hipGetLastError();
  }
  // HumanoidStandup: the Humanoid system lying down, 22 ground rows (F_R2)
  if (fold && L == 16 && (k == BX_ENV_HUMANOID || k == BX_ENV_HUMANOID_STANDUP) &&
      feat == (F_SPH | F_G1 | F_R2)) {
    if (a.packed && a.n_steps <= 1)
      launch_one<EnvArgs>(env_step_packed_kernel<16, 1, F_SPH | F_G1 | F_R2, 8, EK_HUM>, grid, tpb, lds, s, a);
    else
      launch_one<EnvArgs>(env_step_kernel<16, 1, F_SPH | F_G1 | F_R2, 8, EK_HUM>, grid, tpb, lds, s, a);
    return hipGetLastError();
  }
  // every other env's Env.step (one packed step): the one-step kernels, whose
  // first loads need no header
  if (a.packed && a.n_steps <= 1) {
    BX_DISPATCH_SINGLE(env_step_packed_kernel, EnvArgs)
    return hipGetLastError();
  }
  BX_DISPATCH_SINGLE(env_step_kernel, EnvArgs)
  return hipGetLastError();
}
// the joint halves' partner exchange alone (bx_debug_partner)
__global__ void __launch_bounds__(64) partner_kernel(float* out, int lanes) {
  const float v = (float)threadIdx.x;
  out[threadIdx.x] = lanes == 16 ? xh(v) : v;
}
hipError_t debug_partner(float* out64, int lanes, hipStream_t s) {
  hipLaunchKernelGGL(partner_kernel, dim3(1), dim3(64), 0, s, out64, lanes);
  return hipGetLastError();
}
hipError_t debug_stamps(unsigned long long* out, int reset) {
#ifdef BX_STAMPS
  static unsigned long long host[4096][16];
  hipError_t e = hipMemcpyFromSymbol(host, HIP_SYMBOL(bx_stamp_wave), sizeof(host));
  if (reset & 4) {  // the per-workgroup sums themselves (4096 x 16)
    memcpy(out, host, sizeof(host));
    return e;
  }
  for (int k = 0; k < 16; k++) {
    out[k] = 0;
    for (int w = 0; w < 4096; w++) out[k] += host[w][k];
  }
  if (e == hipSuccess && reset) {
    memset(host, 0, sizeof(host));
    e = hipMemcpyToSymbol(HIP_SYMBOL(bx_stamp_wave), host, sizeof(host));
  }
  return e;
#else
  (void)out;
  (void)reset;
  return hipErrorNotSupported;
#endif
}
#else
hipError_t launch_system_step_generic(int L, int mode, int feat, int tpb, int64_t n_envs, size_t lds,
                                      hipStream_t s, const StepArgs& a) {
  const int epb = tpb / L;
  dim3 grid((unsigned)((n_envs + epb - 1) / epb));
  BX_DISPATCH_GENERIC(system_step_kernel, StepArgs)
  return hipGetLastError();
}
hipError_t launch_env_step_generic(int L, int mode, int feat, int tpb, int64_t n_envs, size_t lds,
                                   hipStream_t s, const EnvArgs& a) {
  const int epb = tpb / L;
  dim3 grid((unsigned)((n_envs + epb - 1) / epb));
  BX_DISPATCH_GENERIC(env_step_kernel, EnvArgs)
  return hipGetLastError();
}
hipError_t launch_system_step_multi(int L, int jh, int64_t n_envs, size_t lds, hipStream_t s,
                                    const StepArgs& a) {
  dim3 grid((unsigned)n_envs);
  switch (L * 2 + (jh ? 1 : 0)) {
    case 128 * 2: launch_one<StepArgs>(system_step_multi_kernel<128>, grid, 128, lds, s, a); break;
    case 128 * 2 + 1: launch_one<StepArgs>(system_step_multi_kernel<128, F_JH>, grid, 128, lds, s, a); break;
    case 256 * 2: launch_one<StepArgs>(system_step_multi_kernel<256>, grid, 256, lds, s, a); break;
    case 256 * 2 + 1: launch_one<StepArgs>(system_step_multi_kernel<256, F_JH>, grid, 256, lds, s, a); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}
hipError_t launch_info_obs(int L, int64_t n_envs, size_t lds, hipStream_t s, const InfoArgs& a) {
  int epb = L > 64 ? 1 : 64 / L;
  dim3 grid((unsigned)((n_envs + epb - 1) / epb));
  if (L == 128) { if (lds > 65536) (void)hipFuncSetAttribute((const void*)info_obs_kernel<128>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds); hipLaunchKernelGGL(info_obs_kernel<128>, grid, dim3(128), lds, s, a); }
  else if (L == 256) { if (lds > 65536) (void)hipFuncSetAttribute((const void*)info_obs_kernel<256>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds); hipLaunchKernelGGL(info_obs_kernel<256>, grid, dim3(256), lds, s, a); }
  else if (L == 16) { if (lds > 65536) (void)hipFuncSetAttribute((const void*)info_obs_kernel<16>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds); hipLaunchKernelGGL(info_obs_kernel<16>, grid, dim3(64), lds, s, a); }
  else if (L == 32) { if (lds > 65536) (void)hipFuncSetAttribute((const void*)info_obs_kernel<32>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds); hipLaunchKernelGGL(info_obs_kernel<32>, grid, dim3(64), lds, s, a); }
  else { if (lds > 65536) (void)hipFuncSetAttribute((const void*)info_obs_kernel<64>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds); hipLaunchKernelGGL(info_obs_kernel<64>, grid, dim3(64), lds, s, a); }
  return hipGetLastError();
}
hipError_t debug_mstamps(unsigned long long* out, int reset) {
#ifdef BX_MSTAMPS
  static unsigned long long host[4096][16];
  hipError_t e = hipMemcpyFromSymbol(host, HIP_SYMBOL(bx_mstamp_wave), sizeof(host));
  for (int k = 0; k < 16; k++) {
    out[k] = 0;
    for (int w = 0; w < 4096; w++) out[k] += host[w][k];
  }
  if (e == hipSuccess && reset) {
    memset(host, 0, sizeof(host));
    e = hipMemcpyToSymbol(HIP_SYMBOL(bx_mstamp_wave), host, sizeof(host));
  }
  return e;
#else
  (void)out;
  (void)reset;
  return hipErrorNotSupported;
#endif
}
hipError_t launch_default_qp(int64_t n_envs, size_t lds, hipStream_t s, const ResetArgs& a) {
  dim3 grid((unsigned)((n_envs + 63) / 64));
  if (lds > 65536) (void)hipFuncSetAttribute((const void*)default_qp_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  hipLaunchKernelGGL(default_qp_kernel, grid, dim3(64), lds, s, a);
  return hipGetLastError();
}
hipError_t launch_uniform(float* out, int64_t n, uint64_t seed, uint64_t offset, float lo, float hi,
                          hipStream_t s) {
  dim3 grid((unsigned)((n + 255) / 256));
  hipLaunchKernelGGL(uniform_kernel, grid, dim3(256), 0, s, out, n, seed, offset, lo, hi);
  return hipGetLastError();
}
hipError_t launch_uniform_slabs(float* out, int64_t slab_n, int64_t n_slabs, uint64_t seed,
                                uint64_t offset, uint64_t slab_stride, const int64_t* epoch,
                                uint64_t epoch_stride, float lo, float hi, hipStream_t s) {
  const int64_t n = slab_n * n_slabs;
  dim3 grid((unsigned)((n + 255) / 256));
  hipLaunchKernelGGL(uniform_slabs_kernel, grid, dim3(256), 0, s, out, slab_n, n, seed, offset,
                     slab_stride, epoch, epoch_stride, lo, hi);
  return hipGetLastError();
}

#endif  // BX_TU_FAST

}  // namespace bx
