#include <cstdio>
// bx_capi.cpp — the C ABI (include/brax_amd.h): descriptor -> device blob,
// argument validation, and stream-ordered kernel launches.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <array>
#include <cmath>
#include <cstring>
#include <map>
#include <string>
#include <vector>

#include "../../include/brax_amd.h"
#include "pbd_launch.h"
#include "pbd_layout.h"

using namespace bx;

namespace {

thread_local std::string g_err;

int fail(const std::string& m) {
  g_err = m;
  return 1;
}

#define HIP_OK(expr)                                                       \
  do {                                                                     \
    hipError_t _e = (expr);                                                \
    if (_e != hipSuccess) return fail(std::string(#expr) + ": " + hipGetErrorString(_e)); \
  } while (0)

uint32_t fbits(double x) {
  float f = (float)x;
  uint32_t u;
  std::memcpy(&u, &f, 4);
  return u;
}

// a joint limit l (radians, as the record holds it in float) as the kernels
// test it (pbd_layout.h LL_*): its pseudo-angle (pbd_math.h pseudo_angle, a
// monotone stand-in for atan2 over (-pi, pi]; +-3 at or past +-pi, where no
// angle is out of range) and its cosine / sine, in double
void limit_trig(float lf, double* p, double* c, double* s) {
  const double l = lf;
  *c = std::cos(l);
  *s = std::sin(l);
  if (l <= -M_PI) *p = -3.0;
  else if (l >= M_PI) *p = 3.0;
  else {
    const double r = std::fabs(*c) + std::fabs(*s), t = r > 0 ? *c / r : 1.0;
    *p = *s >= 0 ? 1.0 - t : t - 1.0;
  }
}

}  // namespace

struct bx_system {
  int device = 0;
  BlobHdr hdr{};
  std::vector<uint32_t> host;
  uint32_t* blob = nullptr;
  int L = 16;       // lanes per env
  int min_L = 16;
  int mode = 0;     // MODE_GLOBAL / MODE_SINGLE / MODE_LDS
  int feat = 31;    // F_SPH | F_ANGLE | F_CC | F_TW | F_FORCE used by this system
  int gw = 8;       // gather width (max per-body list length, 4 or 8)
  int tpb = 64;     // threads per workgroup of the step kernels (multiple of L)
  bool single_ok = false;
  bool multi_ok = false;  // MODE_MULTI (3): large pbd scenes, 128 or 256 threads per env
  float* movf = nullptr;  // MULTI: the penetrating contacts past MCBUF, per env (grown on demand)
  int64_t movf_envs = 0;
  int fold = 0;     // every joint j has torque actuator j (the Ant / Humanoid env kernels)
  int jb = 0;       // the joint-halves env kernels may own body copies (JB, build_blob)
  size_t lds_env = 0;    // bytes per block for the per-env kernels
  size_t lds_reset = 0;  // bytes per block for default_qp
};

namespace {

struct Builder {
  std::vector<uint32_t> w;
  int alloc(int n) {
    int o = (int)w.size();
    w.resize(w.size() + (size_t)std::max(n, 0), 0u);
    return o;
  }
  void f(int o, double x) { w[o] = fbits(x); }
  void i(int o, int x) { w[o] = (uint32_t)x; }
};

// the system's feature mask (F_* of pbd_kernels.hip: what its joints,
// actuators, colliders and layout need), which picks its step kernels
static int system_feat(const bx_desc* d, const BlobHdr& H, int L, int J, int K, int G,
                       int max_groups, bool xcol, bool jh_off, bool r2, bool c16, bool r2g) {
  int f = 0;
  for (int j = 0; j < J; j++) if (d->joint_type[j] != BX_JOINT_REVOLUTE) f |= 1;
  for (int a = 0; a < K; a++) if (d->act_type[a] != BX_ACT_TORQUE) f |= 2;
  for (int g = 0; g < G; g++) {
    if (d->col_fn[g] != BX_COL_CAPSULE_PLANE) f |= 4;
    if (!d->col_oneway[g]) f |= 8;
  }
  if (d->n_forces > 0) f |= 16;
  if (max_groups <= 1) f |= 32;  // F_G1: one collider group per body
  if (xcol) f |= 64;             // F_X: extended contact functions
  // F_JH (joint halves, SINGLE mode at 16 lanes): <= 8 revolute joints, each
  // driven by the actuator of the same index
  if (H.single && L == 16 && J <= 8 && K <= 8 && H.act_same && !(f & 1) && !jh_off) f |= 128;
  if (r2) f |= 256;  // F_R2: two contact rows per lane (SINGLE mode, 16 lanes)
  if (H.single && c16) f |= 512;  // F_C16: 16-entry contact gather lists
  if (r2g) f |= 1024;             // F_R2G: one contact function per row slot
  return f;
}

int build_blob(const bx_desc* d, const bx_reset_desc* r, bx_system* S) {
  // A/B knob: BX_NO_JOINT_HALVES=1 keeps one lane per joint
  const bool jh_off = getenv("BX_NO_JOINT_HALVES") && atoi(getenv("BX_NO_JOINT_HALVES"));
  // A/B switch: BX_NO_R2=1 keeps 17-32-row systems at 32 lanes
  const bool r2_off = getenv("BX_NO_R2") && atoi(getenv("BX_NO_R2"));
  const int N = d->n_bodies, J = d->n_joints, K = d->n_actuators, R = d->n_rows, G = d->n_groups;
  if (N <= 0) return fail("descriptor has no bodies");
  if (d->dynamics_mode != BX_DYN_PBD && d->dynamics_mode != BX_DYN_LEGACY_SPRING)
    return fail("unknown dynamics mode");
  if (d->substeps <= 0) return fail("substeps must be positive");
  for (int j = 0; j < J; j++) {
    if (d->joint_body_p[j] < 0 || d->joint_body_p[j] >= N || d->joint_body_c[j] < 0 ||
        d->joint_body_c[j] >= N)
      return fail("joint body index out of range");
    if (d->joint_type[j] != BX_JOINT_REVOLUTE && d->joint_type[j] != BX_JOINT_SPHERICAL &&
        !(d->joint_type[j] == BX_JOINT_UNIVERSAL && d->dynamics_mode == BX_DYN_LEGACY_SPRING))
      return fail("unsupported joint type");
    if (d->dynamics_mode == BX_DYN_LEGACY_SPRING &&
        (!d->joint_stiffness || !d->joint_spring_damping || !d->joint_limit_strength))
      return fail("legacy_spring descriptor needs joint stiffness, spring damping and limit strength");
  }
  for (int a = 0; a < K; a++) {
    if (d->act_joint[a] < 0 || d->act_joint[a] >= J) return fail("actuator joint out of range");
    for (int l = 0; l < 3; l++)
      if (d->act_index[3 * a + l] >= d->action_size) return fail("actuator index out of range");
  }
  for (int x = 0; x < R; x++) {
    if (d->row_body_a[x] < 0 || d->row_body_a[x] >= N || d->row_body_b[x] < 0 ||
        d->row_body_b[x] >= N)
      return fail("contact row body out of range");
    if (d->row_group[x] < 0 || d->row_group[x] >= G) return fail("contact row group out of range");
    int fn = d->col_fn[d->row_group[x]];
    if (fn < BX_COL_CAPSULE_PLANE || fn > BX_COL_HULL_HULL) return fail("unsupported contact function");
    if (fn == BX_COL_HULL_HULL) {
      if (!d->hull_vert || !d->hull_face || !d->hull_norm) return fail("hull rows need the hull arrays");
      for (int k = 0; k < 2; k++) {
        int hx = (int)d->row_ext[16 * x + k];
        if (hx < 0 || hx >= d->n_hull) return fail("hull row index out of range");
      }
      int e = (int)d->row_ext[16 * x + 2];
      if (e < 0 || e > 3) return fail("hull row contact index out of range");
    }
    if (fn >= BX_COL_HEIGHTMAP && !d->row_ext) return fail("extended contact rows need row_ext");
    if (fn == BX_COL_HEIGHTMAP) {
      if (!d->row_hm || !d->hm_data) return fail("height map rows need row_hm and hm_data");
      int off = d->row_hm[2 * x], m = d->row_hm[2 * x + 1];
      if (m < 2 || off < 0 || (int64_t)off + (int64_t)m * m > d->n_hm)
        return fail("height map row out of range");
    }
  }
  for (int f = 0; f < d->n_forces; f++) {
    if (d->force_body[f] < 0 || d->force_body[f] >= N) return fail("force body out of range");
    if (d->force_type[f] != BX_FORCE_THRUSTER && d->force_type[f] != BX_FORCE_TWISTER)
      return fail("unknown force type");
    if (f > 0 && d->force_type[f] < d->force_type[f - 1])
      return fail("forces must be ordered Thrusters, then Twisters");
  }
  if (G >= 128) return fail("too many collider groups");
  // rows of a group are contiguous; a culled group's rows are in flat order
  for (int x = 1; x < R; x++)
    if (d->row_group[x] < d->row_group[x - 1]) return fail("contact rows must be grouped");
  for (int g = 0; g < G; g++) {
    if (d->col_cutoff[g] < 0) return fail("negative collider cutoff");
    if (d->col_cutoff[g] == 0) continue;
    if (d->col_fn[g] != BX_COL_CAPSULE_CAPSULE) return fail("culling is capsule-capsule only");
    int n = 0, last = -1;
    for (int x = 0; x < R; x++) {
      if (d->row_group[x] != g) continue;
      // a masked cell ranks after every allowed one: only where cutoff needs it
      if (d->row_flat[x] <= last) return fail("culled rows must be in increasing flat order");
      last = d->row_flat[x];
      n++;
    }
    if (d->col_cutoff[g] > n) return fail("collider cutoff exceeds the group's rows");
  }
  if (d->row_nn_masked)
    for (int x = 0; x < R; x++)
      if (d->row_nn_masked[x] && !d->col_cutoff[d->row_group[x]])
        return fail("masked NearNeighbors rows belong to culled groups");
  if (2 * R >= (1 << 24)) return fail("too many contact rows");

  Builder B;
  int o_hdr = B.alloc((int)(sizeof(BlobHdr) / 4));
  (void)o_hdr;
  BlobHdr H{};
  H.N = N; H.J = J; H.K = K; H.R = R; H.G = G; H.A = d->action_size; H.substeps = d->substeps;
  H.num_joint_dof = d->num_joint_dof;
  H.h = (float)d->h;
  H.dt = (float)d->dt;
  // integrators.py:87,91 — exp(damping * dt) of Python doubles, one constant
  H.vexp = (float)std::exp(d->velocity_damping * d->h);
  H.aexp = (float)std::exp(d->angular_damping * d->h);
  H.spring = d->dynamics_mode == BX_DYN_LEGACY_SPRING ? 1 : 0;
  H.gx = (float)d->gravity[0]; H.gy = (float)d->gravity[1]; H.gz = (float)d->gravity[2];

  H.o_body = B.alloc(N * BODY_STRIDE);
  for (int b = 0; b < N; b++) {
    int o = H.o_body + b * BODY_STRIDE;
    B.f(o + BODY_MASS, d->body_mass[b]);
    for (int k = 0; k < 3; k++) {
      B.f(o + BODY_I + k, d->body_inv_inertia[3 * b + k]);
      B.f(o + BODY_PM + k, d->pos_mask[3 * b + k]);
      B.f(o + BODY_RM + k, d->rot_mask[3 * b + k]);
    }
    for (int k = 0; k < 4; k++) B.f(o + BODY_QM + k, d->quat_mask[4 * b + k]);
  }
  H.o_joint = B.alloc(J * JOINT_STRIDE);
  int D = 0;
  for (int j = 0; j < J; j++) {
    int o = H.o_joint + j * JOINT_STRIDE;
    int type = d->joint_type[j];
    // angle_vel dofs (joints.py:218-225): the free dofs of a sphericalised
    // group, else every dof of the joint (1 / 2 / 3)
    int nang = d->joint_free_dofs[j] >= 0 ? d->joint_free_dofs[j] : d->joint_dof[j];
    B.i(o + J_TYPE, type);
    B.i(o + J_BP, d->joint_body_p[j]);
    B.i(o + J_BC, d->joint_body_c[j]);
    B.i(o + J_FREE, d->joint_free_dofs[j]);
    B.i(o + J_DOF, d->joint_dof[j]);
    B.i(o + J_ANGLE_OFF, D);
    B.i(o + J_NANGLES, nang);
    D += nang;
    B.f(o + J_DAMP, d->joint_damping[j]);
    B.f(o + J_SP, d->joint_scale_pos[j]);
    B.f(o + J_SA, d->joint_scale_ang[j]);
    for (int k = 0; k < 3; k++) {
      B.f(o + J_OFFP + k, d->joint_off_p[3 * j + k]);
      B.f(o + J_OFFC + k, d->joint_off_c[3 * j + k]);
    }
    for (int k = 0; k < 9; k++) {
      B.f(o + J_AXP + k, d->joint_axis_p[9 * j + k]);
      B.f(o + J_AXC + k, d->joint_axis_c[9 * j + k]);
    }
    for (int k = 0; k < 6; k++) B.f(o + J_LIM + k, d->joint_limit[6 * j + k]);
    // the limit rows' pseudo-angles and cos / sin (J_JLIM, LL_*), from the
    // radians just stored as float
    for (int row = 0; row < 3; row++)
      for (int side = 0; side < 2; side++) {
        float lf;
        std::memcpy(&lf, &B.w[o + J_LIM + 2 * row + side], 4);
        double p, c, sn;
        limit_trig(lf, &p, &c, &sn);
        const int r = o + J_JLIM + 8 * row;
        B.f(r + (side ? LL_PHI : LL_PLO), p);
        B.f(r + (side ? LL_CHI : LL_CLO), c);
        B.f(r + (side ? LL_SHI : LL_SLO), sn);
      }
    if (d->dynamics_mode == BX_DYN_LEGACY_SPRING) {
      B.f(o + J_STIFF, d->joint_stiffness[j]);
      B.f(o + J_SDAMP, d->joint_spring_damping[j]);
      B.f(o + J_LSTR, d->joint_limit_strength[j]);
    }
  }
  H.D = D;
  H.o_act = B.alloc(K * ACT_STRIDE);
  for (int a = 0; a < K; a++) {
    int o = H.o_act + a * ACT_STRIDE;
    B.i(o + A_TYPE, d->act_type[a]);
    B.i(o + A_JOINT, d->act_joint[a]);
    for (int k = 0; k < 3; k++) B.i(o + A_IDX + k, d->act_index[3 * a + k]);
    B.f(o + A_STR, d->act_strength[a]);
  }
  H.o_row = B.alloc(R * ROW_STRIDE);
  for (int x = 0; x < R; x++) {
    int o = H.o_row + x * ROW_STRIDE;
    int g = d->row_group[x];
    B.i(o + R_GROUP, g);
    B.i(o + R_A, d->row_body_a[x]);
    B.i(o + R_B, d->row_body_b[x]);
    B.i(o + R_FN, d->col_fn[g]);
    B.i(o + R_ONEWAY, d->col_oneway[g]);
    for (int k = 0; k < 3; k++) {
      B.f(o + R_APOS + k, d->row_a_pos[3 * x + k]);
      B.f(o + R_AEND + k, d->row_a_end[3 * x + k]);
      B.f(o + R_BPOS + k, d->row_b_pos[3 * x + k]);
      B.f(o + R_BEND + k, d->row_b_end[3 * x + k]);
    }
    B.f(o + R_ARAD, d->row_a_radius[x]);
    B.f(o + R_BRAD, d->row_b_radius[x]);
    B.f(o + R_FRIC, d->row_friction[x]);
    B.f(o + R_ELAS, d->row_elasticity[x]);
    B.f(o + R_SCALE, d->col_scale[g]);
    B.f(o + R_THR, d->col_velocity_threshold[g]);
    B.f(o + R_ERP, d->col_baumgarte_erp[g]);
    if (d->row_ext)
      for (int k = 0; k < 16; k++) B.f(o + R_X + k, d->row_ext[16 * x + k]);
    B.i(o + R_NNMASK, d->row_nn_masked && d->row_nn_masked[x] ? 1 : 0);
    B.i(o + R_FLAT, d->col_cutoff[g] ? d->row_flat[x] : -1);
    if (d->col_fn[g] == BX_COL_HEIGHTMAP) {
      B.i(o + R_HM_OFF, d->row_hm[2 * x]);
      B.i(o + R_HM_M, d->row_hm[2 * x + 1]);
    }
  }
  H.o_hm = B.alloc(d->n_hm > 0 ? d->n_hm : 0);
  for (int k = 0; k < d->n_hm; k++) B.f(H.o_hm + k, d->hm_data[k]);
  H.o_hull = B.alloc(d->n_hull > 0 ? d->n_hull * HULL_STRIDE : 0);
  for (int h = 0; h < d->n_hull; h++) {
    int o = H.o_hull + h * HULL_STRIDE;
    for (int k = 0; k < 24; k++) B.f(o + HULL_V + k, d->hull_vert[24 * h + k]);
    for (int k = 0; k < 72; k++) B.f(o + HULL_F + k, d->hull_face[72 * h + k]);
    for (int k = 0; k < 18; k++) B.f(o + HULL_N + k, d->hull_norm[18 * h + k]);
  }
  // collider groups: cutoff, row range, Info base (system.py:36-43 order)
  H.o_group = B.alloc(G * GROUP_STRIDE);
  {
    int info = 0;
    for (int g = 0; g < G; g++) {
      int r0 = R, r1 = 0;
      for (int x = 0; x < R; x++)
        if (d->row_group[x] == g) { r0 = std::min(r0, x); r1 = std::max(r1, x + 1); }
      if (r0 > r1) r0 = r1 = 0;
      int o = H.o_group + g * GROUP_STRIDE;
      B.i(o + G_CUT, d->col_cutoff[g]);
      B.i(o + G_R0, r0);
      B.i(o + G_R1, r1);
      B.i(o + G_INFO, info);
      info += d->col_cutoff[g] ? d->col_cutoff[g] : r1 - r0;
      if (d->col_cutoff[g]) H.n_nn++;
    }
    H.info_rows = info;
  }
  H.NF = d->n_forces;
  H.o_force = B.alloc(d->n_forces * FORCE_STRIDE);
  for (int f = 0; f < d->n_forces; f++) {
    int o = H.o_force + f * FORCE_STRIDE;
    B.i(o + F_TYPE, d->force_type[f]);
    B.i(o + F_BODY, d->force_body[f]);
    for (int k = 0; k < 3; k++) B.i(o + F_IDX + k, d->force_index[3 * f + k]);
    B.f(o + F_STR, d->force_strength[f]);
    B.f(o + F_MASS, d->body_mass[d->force_body[f]]);
  }
  // gather lists (the reference's segment_sum order: per group, parents then
  // children / a-rows then b-rows)
  std::vector<std::vector<int>> jl(N), al(N), cl(N);
  for (int j0 = 0; j0 < J;) {
    int g = d->joint_group[j0], j1 = j0;
    while (j1 < J && d->joint_group[j1] == g) j1++;
    for (int j = j0; j < j1; j++) jl[d->joint_body_p[j]].push_back(j);
    for (int j = j0; j < j1; j++) jl[d->joint_body_c[j]].push_back(J + j);
    j0 = j1;
  }
  for (int a0 = 0; a0 < K;) {
    int g = d->act_group[a0], a1 = a0;
    while (a1 < K && d->act_group[a1] == g) a1++;
    for (int a = a0; a < a1; a++) al[d->joint_body_p[d->act_joint[a]]].push_back(a);
    for (int a = a0; a < a1; a++) al[d->joint_body_c[d->act_joint[a]]].push_back(K + a);
    a0 = a1;
  }
  for (int g = 0; g < G; g++) {
    for (int x = 0; x < R; x++)
      if (d->row_group[x] == g) cl[d->row_body_a[x]].push_back(x | (g << 24));
    if (!d->col_oneway[g])
      for (int x = 0; x < R; x++)
        if (d->row_group[x] == g) cl[d->row_body_b[x]].push_back((R + x) | (g << 24));
  }
  auto put_lists = [&](std::vector<std::vector<int>>& L_, int& o_off, int& o_l) {
    o_off = B.alloc(N + 1);
    int tot = 0;
    for (int b = 0; b < N; b++) tot += (int)L_[b].size();
    o_l = B.alloc(tot);
    int k = 0;
    for (int b = 0; b < N; b++) {
      B.i(o_off + b, k);
      for (int v : L_[b]) B.i(o_l + k++, v);
    }
    B.i(o_off + N, k);
  };
  put_lists(jl, H.o_jl_off, H.o_jl);
  put_lists(al, H.o_al_off, H.o_al);
  put_lists(cl, H.o_cl_off, H.o_cl);
  // MULTI-mode gather tasks: each body's contact list cut, per collider group,
  // into runs of <= TASK_W entries (same order); a body's tasks in list order.
  // An entry names a row and side (row | side << 15, pbd_layout.h MCAP):
  // the kernel finds the side's slot through the row's compact index; the
  // padding entry is row R (never indexed); the zero slot is 2 MCAP
  H.m_zero = 2 * MCAP;
  auto mslot_of = [&](int s) { return s < R ? s : ((s - R) | 0x8000); };
  std::vector<std::vector<int>> task_e;  // row | side << 15
  std::vector<std::vector<int>> btask(N);  // task | group << 24
  int max_btask = 0;
  for (int b = 0; b < N; b++) {
    size_t i = 0;
    while (i < cl[b].size()) {
      const int g = cl[b][i] >> 24;
      std::vector<int> t;
      while (i < cl[b].size() && (cl[b][i] >> 24) == g && (int)t.size() < TASK_W)
        t.push_back(mslot_of(cl[b][i++] & 0xFFFFFF));
      btask[b].push_back((int)task_e.size() | (g << 24));
      task_e.push_back(t);
    }
    max_btask = std::max(max_btask, (int)btask[b].size());
  }
  H.T = (int)task_e.size();
  H.o_task = B.alloc(H.T * TASK_W);
  for (int t = 0; t < H.T; t++)
    for (int k = 0; k < TASK_W; k++)
      B.i(H.o_task + t * TASK_W + k, k < (int)task_e[t].size() ? task_e[t][k] : R);
  H.o_btask = B.alloc(N * BTASK_W);
  for (int b = 0; b < N; b++) {
    // padding: the zero task (index T, a zero partial) in the last group
    const int gl = btask[b].empty() ? 0 : (btask[b].back() >> 24);
    for (int k = 0; k < BTASK_W; k++)
      B.i(H.o_btask + b * BTASK_W + k,
          k < (int)btask[b].size() ? btask[b][k] : (H.T | (gl << 24)));
  }

  // reset tables
  if (r) {
    H.n_fk = r->n_fk;
    H.n_root_groups = r->n_root_groups;
    H.o_base = B.alloc(N * 13);
    for (int k = 0; k < N * 13; k++) B.f(H.o_base + k, r->base_qp[k]);
    H.o_fk = B.alloc(r->n_fk * FK_STRIDE);
    for (int f = 0; f < r->n_fk; f++) {
      int o = H.o_fk + f * FK_STRIDE;
      if (r->fk_body_p[f] < 0 || r->fk_body_p[f] >= N || r->fk_body_c[f] < 0 || r->fk_body_c[f] >= N)
        return fail("reset joint body out of range");
      B.i(o + FK_BP, r->fk_body_p[f]);
      B.i(o + FK_BC, r->fk_body_c[f]);
      for (int l = 0; l < 3; l++) {
        int ix = r->fk_dof_index[3 * f + l];
        if (ix >= d->num_joint_dof) return fail("reset dof index out of range");
        B.i(o + FK_IDX + l, ix);
      }
      for (int k = 0; k < 4; k++) {
        B.f(o + FK_ROT + k, r->fk_rot[4 * f + k]);
        B.f(o + FK_REF + k, r->fk_ref[4 * f + k]);
      }
      for (int k = 0; k < 3; k++) {
        B.f(o + FK_OFFP + k, r->fk_off_p[3 * f + k]);
        B.f(o + FK_OFFC + k, r->fk_off_c[3 * f + k]);
      }
    }
    std::vector<std::vector<int>> zl(N);
    for (int p = 0; p < r->n_zpts; p++) {
      if (r->zpt_body[p] < 0 || r->zpt_body[p] >= N) return fail("min_z point body out of range");
      zl[r->zpt_body[p]].push_back(p);
    }
    H.o_zoff = B.alloc(N + 1);
    H.o_zpt = B.alloc(r->n_zpts * 4);
    int k = 0;
    for (int b = 0; b < N; b++) {
      B.i(H.o_zoff + b, k);
      for (int p : zl[b]) {
        for (int q = 0; q < 3; q++) B.f(H.o_zpt + 4 * k + q, r->zpt_local[3 * p + q]);
        B.f(H.o_zpt + 4 * k + 3, r->zpt_radius[p]);
        k++;
      }
    }
    B.i(H.o_zoff + N, k);
    H.o_dangle = B.alloc(d->num_joint_dof);
    for (int k = 0; k < d->num_joint_dof; k++)
      B.f(H.o_dangle + k, r->default_angle ? r->default_angle[k] : 0.0);
    H.o_zero = B.alloc(N);
    H.o_rgroup = B.alloc(N);
    for (int b = 0; b < N; b++) {
      B.i(H.o_zero + b, r->body_zero_cand[b]);
      B.i(H.o_rgroup + b, r->body_root_group[b]);
    }
  }
  H.const_words = (((r ? H.o_base : (int)B.w.size())) + 3) & ~3;

  // the register-hoisted (SINGLE) kernels' shape limits, independent of the
  // lane count: gather lists of <= 8 entries, <= 2 collider groups per body,
  // the pbd step without culling or the extended contact functions
  size_t mx = 0;
  int max_groups = 0;
  bool xcol = false;  // extended contact functions run in the item-loop kernel
  for (int g = 0; g < G; g++) xcol |= d->col_fn[g] >= BX_COL_HEIGHTMAP;
  for (int b = 0; b < N; b++) {
    mx = std::max({mx, jl[b].size(), al[b].size(), cl[b].size()});
    std::vector<int> gs;
    for (int v : cl[b])
      if (std::find(gs.begin(), gs.end(), v >> 24) == gs.end()) gs.push_back(v >> 24);
    max_groups = std::max(max_groups, (int)gs.size());
  }
  // F_C16: a body's contact list may hold up to 16 entries (its joint and
  // actuator lists <= 8), the SINGLE kernels then gather 16 contact slots
  size_t mx_ja = 0, mx_c = 0;
  for (int b = 0; b < N; b++) {
    mx_ja = std::max({mx_ja, jl[b].size(), al[b].size()});
    mx_c = std::max(mx_c, cl[b].size());
  }
  const bool c16 = mx_c > 8 && mx_c <= 16 && mx_ja <= 8;
  const bool single_shape = (mx <= 8 || c16) && max_groups <= 2 && H.n_nn == 0 &&
                            d->dynamics_mode != BX_DYN_LEGACY_SPRING && !xcol;
  // per-env LDS layout
  int L = std::max({N, J, K, R, 1});
  // an env is one 16/32/64-lane segment of a wave; past 64 items (large
  // scenes) it spreads over a whole 128- or 256-thread workgroup
  L = L <= 16 ? 16 : L <= 32 ? 32 : L <= 64 ? 64 : L <= 128 ? 128 : 256;
  // 17-32 contact rows and <= 16 bodies / joints / actuators: SINGLE mode at
  // 16 lanes with two rows per lane (F_R2: rows l and l + 16), not 32 lanes
  // for the rows alone (HalfCheetah, HumanoidStandup, Fetch)
  const bool r2 = L == 32 && std::max({N, J, K}) <= 16 && R <= 32 && single_shape && !r2_off;
  if (r2) L = 16;
  H.L = L;
  int off = 0;
  auto carve = [&](int n) { int o = off; off += (n + 3) & ~3; return o; };
  H.l_qp = carve(N * QP_STRIDE);
  H.l_prev = carve(N * PREV_STRIDE);
  H.l_rb = carve(N * RB_STRIDE);
  // slot regions end with one zero slot (padding target of the gather lists)
  H.l_jslot = carve((2 * J + 1) * SLOT_STRIDE);
  H.l_aslot = carve((2 * K + 1) * ASLOT_STRIDE);
  // the active-row list: culled scenes only (the SINGLE kernels never cull;
  // MULTI's all-pairs scenes need the room)
  H.l_alist = carve(H.n_nn ? H.info_rows : 0);
  H.l_red = carve(64);
  // NearNeighbors: each wave's sorted picks (64-bit keys) when an env spans
  // up to 4 waves (carved with the env-step regions below; the MULTI kernel
  // keeps them in its task-partials region)
  {
    int max_cut = 0;
    for (int g = 0; g < G; g++) max_cut = std::max(max_cut, d->col_cutoff[g]);
    H.nnl_words = 2 * 4 * max_cut;
  }
  // the MULTI kernel's row tables: the rows' collidables as the distinct
  // (body, offset, end, radius) records, whose centres the broad phase and
  // the NearNeighbors keys place in the world once per pass (culled scenes:
  // once per step) for every row naming them, and from which the contact
  // passes assemble a row's geometry in LDS
  std::map<std::array<uint32_t, 8>, int> cen_ix;
  std::vector<std::array<uint32_t, 8>> cens;
  std::vector<int> row_cen(2 * R, 0);
  // and the rows' impulse constants as the distinct (friction, elasticity,
  // scale, velocity threshold) materials
  std::map<std::array<uint32_t, 4>, int> mat_ix;
  std::vector<std::array<uint32_t, 4>> mats;
  std::vector<int> row_mat(R, 0);
  for (int x = 0; x < R; x++) {
    // (the row record's words: the bits the row image carried)
    const uint32_t* w = &B.w[H.o_row + x * ROW_STRIDE];
    for (int side = 0; side < 2; side++) {
      const int o = side ? R_BPOS : R_APOS, oe = side ? R_BEND : R_AEND, orr = side ? R_BRAD : R_ARAD;
      const std::array<uint32_t, 8> k{w[side ? R_B : R_A], w[o], w[o + 1], w[o + 2],
                                      w[oe], w[oe + 1], w[oe + 2], w[orr]};
      auto it = cen_ix.find(k);
      if (it == cen_ix.end()) {
        it = cen_ix.emplace(k, (int)cens.size()).first;
        cens.push_back(k);
      }
      row_cen[2 * x + side] = it->second;
    }
    const std::array<uint32_t, 4> m{w[R_FRIC], w[R_ELAS], w[R_SCALE], w[R_THR]};
    auto it = mat_ix.find(m);
    if (it == mat_ix.end()) {
      it = mat_ix.emplace(m, (int)mats.size()).first;
      mats.push_back(m);
    }
    row_mat[x] = it->second;
  }
  // (past these sizes the scene takes the item-loop kernels: no MULTI tables)
  const bool mtab_ok = cens.size() <= 256 && mats.size() <= 0xFF && R <= 0xFFFF;
  H.n_cen = mtab_ok ? (int)cens.size() : 0;
  H.n_mat = mtab_ok ? (int)mats.size() : 0;
  // the MULTI (System.step only) tail starts here, over the env step's regions
  const int tail_m = off;
  // env-step regions: joint angles, the env programs' System.step action
  // (swimmer: + drag, grasp: 3 palm actions), the staged action row (every
  // index an actuator or force reads: jp.take clips into the row, so no read
  // lands past these words)
  // (the Info accumulators and the NearNeighbors ranks: the MULTI kernel
  // keeps them in its contact slots / contact buffer, dead when these live)
  H.l_acc = carve(N * ACC_STRIDE);
  H.l_ract = carve(H.n_nn ? R : 0);
  H.l_nnl = carve(H.nnl_words);
  H.l_ang = carve(2 * D);
  H.xact_words = std::max(16, (d->action_size + 12 + 3) & ~3);
  H.l_xact = carve(H.xact_words);
  H.act_read = std::max(d->action_size, 1);
  for (int k = 0; k < 3 * K; k++) H.act_read = std::max(H.act_read, d->act_index[k] + 1);
  for (int k = 0; k < 3 * d->n_forces; k++) H.act_read = std::max(H.act_read, d->force_index[k] + 1);
  H.l_arow = carve(H.act_read);
  // the contact regions form each mode's tail: the item-loop / SINGLE
  // kernels keep per-row data and 12-word slots, MULTI mode keeps the row data
  // in registers and needs 6-word slots plus the task partials
  const int tail = off;
  off = tail_m;
  // the chunk's contact slots (2 MCAP + the zero slot; the Info accumulators
  // alias them after the substeps)
  H.l_mslot = carve(std::max((2 * MCAP + 1) * MSLOT_STRIDE, N * ACC_STRIDE));
  // the task partials; before the passes read them the same words hold the
  // broad phase's near-row list (16-bit), the NearNeighbors pick lists and the
  // serial picks' distances
  H.l_tslot = carve(std::max({(H.T + 1) * TSLOT_STRIDE, (R + 1) / 2, H.nnl_words, H.n_nn ? R : 0}));
  H.l_near = H.l_tslot;
  H.l_cnt = carve(48);
  H.l_nearc = H.l_cnt;
  // the rows' compact contact indices (16-bit, R + 1: the padding row R)
  H.l_sidx = carve((R + 2) / 2);
  // the penetrating rows' contacts, then their rows (16-bit)
  H.l_cbuf = carve(std::max(MCBUF * MCB_W + MCBUF / 2, H.n_nn ? R : 0));
  // the broad phase's row bounds and centres (constants, then world), staged
  // once per launch
  H.l_bimg = carve(BI_WORDS * R);
  H.l_cen = carve(4 * (3 * H.n_cen + H.n_mat + N));
  H.env_words_m = (off + 63) & ~63;
  if (getenv("BX_PLAN_DEBUG"))
    fprintf(stderr,
            "bx plan (words): qp..red %d  mslot %d  tslot %d (T=%d)  cnt+sidx+cbuf %d  bimg %d  "
            "cen %d (n_cen=%d n_mat=%d)  ract %d  alist %d  nnl %d  env_words_m %d (%d B)\n",
            H.l_red + 64, H.l_tslot - H.l_mslot, H.l_cnt - H.l_tslot, H.T, H.l_bimg - H.l_cnt,
            H.l_cen - H.l_bimg, 4 * (3 * H.n_cen + H.n_mat + N), H.n_cen, H.n_mat,
            H.n_nn ? R : 0, H.n_nn ? H.info_rows : 0, H.nnl_words, H.env_words_m, 4 * H.env_words_m);
  off = tail;
  H.l_rowd = carve(R * ROWD_STRIDE);
  H.l_cslot = carve((2 * R + 1) * SLOT_STRIDE);
  // SINGLE mode: the spherical kernels' joint limit rows, staged from the
  // lane image once per launch (6 16-byte groups per lane, LIM_SLOTS; sized
  // for this system's L, which bx_system_set_variant keeps)
  const bool single_fit = N <= L && J <= L && K <= L && (R <= L || r2) && single_shape &&
                          (mx <= 8 || L == 16);
  // (carved below, once the features say the system's SINGLE kernel reads it)
  const int jlim_at = off;
  H.l_jlim = 0;
  // envs 64 words apart: with the odd-multiple record strides, the four
  // envs' records of one ds_read_b128 lane group land on distinct bank slots
  H.env_words = (off + 63) & ~63;
  {
    // the register-hoisted kernel is the pbd step only; legacy_spring systems
    // run the item-loop kernel
    H.single = single_fit ? 1 : 0;  // F_C16 kernels: 16 lanes
    // MULTI mode: a pbd scene past one wave (256 threads per env), every
    // lane owning <= 1 body / joint / actuator / task and <= MULTI_MR rows
    size_t mxja = 0;
    for (int b = 0; b < N; b++) mxja = std::max({mxja, jl[b].size(), al[b].size()});
    // (and its LDS tail within one workgroup's 160 KB)
    H.multi = (!H.single && L > 64 && !H.spring && !xcol && N <= 256 && J <= 256 && K <= 256 &&
               H.T <= 2 * 256 && G < 64 && R <= 8 * 256 && mxja <= 8 && max_btask <= BTASK_W && mtab_ok &&
               (size_t)H.env_words_m * 4 <= 160 * 1024) ? 1 : 0;
    H.act_same = 1;
    for (int a = 0; a < K; a++)
      if (d->act_joint[a] != a) H.act_same = 0;
  }
  // JB's body conditions (the env kernels whose joint-halves lanes own body
  // copies): every body on no joint side is frozen in all dimensions
  // (position, rotation and the quaternion's vector part masks zero) and
  // touches contact rows only as the plane side of one-way rows (its record
  // then never changes and its contact sums are zeros)
  auto jb_bodies_ok = [&]() {
    std::vector<char> side(N, 0);
    for (int j = 0; j < J; j++) side[d->joint_body_p[j]] = side[d->joint_body_c[j]] = 1;
    for (int b = 0; b < N; b++) {
      if (side[b]) continue;
      const uint32_t* bw = &B.w[H.o_body + b * BODY_STRIDE];
      for (int k = 0; k < 3; k++)
        if (bw[BODY_PM + k] != fbits(0.0) || bw[BODY_RM + k] != fbits(0.0)) return false;
      // (the reference's quaternion mask keeps w at 1 for a frozen rotation:
      // integrators.py's [0] + frozen.rotation; the w update is an exact zero)
      for (int k = 1; k < 4; k++)
        if (bw[BODY_QM + k] != fbits(0.0)) return false;
    }
    for (int x = 0; x < R; x++) {
      if (!side[d->row_body_a[x]]) return false;
      if (!side[d->row_body_b[x]] && !d->col_oneway[d->row_group[x]]) return false;
    }
    return true;
  };
  const int HB = 8;  // the joint halves' half width (lanes per side)
  // a contact row's 32 resolved words (LR_*): its record's geometry and
  // constants with the masses / inverse inertias of the bodies it names
  auto row_words = [&](int x, uint32_t* out) {
    const uint32_t* w = &B.w[H.o_row + x * ROW_STRIDE];
    const uint32_t* pa = &B.w[H.o_body + (int)w[R_A] * BODY_STRIDE];
    const uint32_t* pb = &B.w[H.o_body + (int)w[R_B] * BODY_STRIDE];
    const int src[24] = {R_GROUP, R_A, R_B, R_FN, R_ONEWAY, R_APOS, R_APOS + 1, R_APOS + 2,
                         R_AEND, R_AEND + 1, R_AEND + 2, R_ARAD, R_BPOS, R_BPOS + 1, R_BPOS + 2,
                         R_BEND, R_BEND + 1, R_BEND + 2, R_BRAD, R_FRIC, R_ELAS, R_SCALE, R_THR,
                         R_ERP};
    for (int k = 0; k < 24; k++) out[k] = w[src[k]];
    out[LR_MA] = pa[BODY_MASS];
    out[LR_MB] = pb[BODY_MASS];
    for (int k = 0; k < 3; k++) {
      out[LR_IA + k] = pa[BODY_I + k];
      out[LR_IB + k] = pb[BODY_I + k];
    }
  };
  // the MULTI kernel's row tables (BI_*: bounds / flags per row; collidables,
  // materials and bodies after them)
  if (H.multi && R > 0) {
    B.alloc((4 - (int)B.w.size() % 4) % 4);  // 16-byte aligned groups
    // broad-phase bounds (BI_*): reach = |a_end| + |b_end| + radii in double,
    // rounded up to float
    std::vector<uint32_t> bimg(BI_WORDS * R, 0u);
    for (int x = 0; x < R; x++) {
      const int g = d->row_group[x];
      double reach = d->row_a_radius[x] + d->row_b_radius[x];
      double ea = 0, eb = 0;
      for (int k = 0; k < 3; k++) {
        ea += d->row_a_end[3 * x + k] * d->row_a_end[3 * x + k];
        eb += d->row_b_end[3 * x + k] * d->row_b_end[3 * x + k];
      }
      reach += std::sqrt(ea) + std::sqrt(eb);
      // the broad phase compares squared centre distances with (reach +
      // 1e-4)^2, rounded up (the margin far above the fp32 error of the
      // centres; a row it keeps that cannot touch only costs its test)
      const double r2 = (reach + 1e-4) * (reach + 1e-4);
      // as a half float rounded up (+inf past 65504: always near)
      uint16_t hb = 0x7C00u;
      if (r2 <= 65504.0) {
        hb = __builtin_bit_cast(uint16_t, (_Float16)r2);
        if ((double)__builtin_bit_cast(_Float16, hb) < r2) hb++;
      }
      uint32_t* bw = &bimg[BI_WORDS * x];
      const bool skip = d->col_fn[g] == BX_COL_CAPSULE_CAPSULE;
      const bool cull = d->col_cutoff[g] != 0;
      uint32_t fl = (skip ? BIF_SKIP : 0u) | (cull ? BIF_CULL : 0u) |
                    (d->row_nn_masked && d->row_nn_masked[x] ? BIF_MASK : 0u) |
                    (d->col_oneway[g] ? BIF_OW : 0u) | ((uint32_t)d->col_fn[g] << BIF_FN_SHIFT) |
                    ((uint32_t)row_mat[x] << BIF_MAT_SHIFT);
      uint32_t info = 0u;
      if (!cull) {
        // the unculled row's Info index (its group's first Info row + its offset)
        const int og = H.o_group + g * GROUP_STRIDE;
        info = (uint32_t)((int)B.w[og + G_INFO] + x - (int)B.w[og + G_R0]);
      }
      bw[BI_W0] = (uint32_t)row_cen[2 * x] | ((uint32_t)row_cen[2 * x + 1] << 8) | (fl << 16);
      bw[BI_W1] = (uint32_t)hb | (info << 16);
    }
    H.o_bimg = B.alloc(BI_WORDS * R);
    for (int k = 0; k < BI_WORDS * R; k++) B.w[H.o_bimg + k] = bimg[k];
    B.alloc((4 - (int)B.w.size() % 4) % 4);  // 16-byte aligned groups
    H.o_cen = B.alloc(8 * H.n_cen + 4 * H.n_mat + 4 * N);
    for (int k = 0; k < H.n_cen; k++)
      for (int i = 0; i < 8; i++) B.w[H.o_cen + 8 * k + i] = cens[k][i];
    const int o_mat = H.o_cen + 8 * H.n_cen, o_bod = o_mat + 4 * H.n_mat;
    for (int k = 0; k < H.n_mat; k++)
      for (int i = 0; i < 4; i++) B.w[o_mat + 4 * k + i] = mats[k][i];
    // the bodies' (mass, inverse inertia), the rows' ma / Ia / mb / Ib
    for (int b = 0; b < N; b++) {
      B.w[o_bod + 4 * b] = B.w[H.o_body + b * BODY_STRIDE + BODY_MASS];
      for (int i = 0; i < 3; i++) B.w[o_bod + 4 * b + 1 + i] = B.w[H.o_body + b * BODY_STRIDE + BODY_I + i];
    }
  }
  // the SINGLE-mode lane image (pbd_layout.h LI_*): copies of the records
  // above, so its words are the same bits the item-loop kernels read; a lane
  // without an item of a kind gets item 0's record (as the kernels' clamped
  // index did), and zeros where the system has none of that kind
  // F_R2: which rows each lane works. Rows of one contact function share a
  // slot where they fit (HalfCheetah, Pusher: the plane rows in the first,
  // the capsule-capsule rows in the second), so a pass runs one function per
  // slot instead of both on every lane; otherwise rows l and l + 16
  std::vector<int> slot1(16, -1), slot2(16, -1);
  bool r2g = false;  // F_R2G: slot 1 one-way capsule-plane, slot 2 two-way capsule-capsule
  if (r2) {
    std::vector<int> pl, other;
    for (int x = 0; x < R; x++)
      (d->col_fn[d->row_group[x]] == BX_COL_CAPSULE_PLANE ? pl : other).push_back(x);
    if (!pl.empty() && !other.empty() && pl.size() <= 16 && other.size() <= 16) {
      r2g = true;
      for (int x : pl) r2g &= d->col_oneway[d->row_group[x]] != 0;
      for (int x : other)
        r2g &= d->col_fn[d->row_group[x]] == BX_COL_CAPSULE_CAPSULE && !d->col_oneway[d->row_group[x]];
      // F_R2G's two-way slot runs as contact halves: row k's a side on lane
      // k, its b side on lane k + 8 (pbd_kernels.hip position_contact_half)
      r2g &= other.size() <= 8;
      for (size_t i = 0; i < pl.size(); i++) slot1[i] = pl[i];
      for (size_t i = 0; i < other.size(); i++) {
        slot2[i] = other[i];
        if (r2g) slot2[i + 8] = other[i];
      }
    } else {
      for (int l = 0; l < 16; l++) {
        slot1[l] = l < R ? l : -1;
        slot2[l] = l + 16 < R ? l + 16 : -1;
      }
    }
  }
  // records in the lane images' layouts, each word through put(lane, word,
  // value): a joint (LJ_*, with its bodies' masses / inverse inertias), its
  // limit row `row` (LL_*: pseudo-angles and cos / sin, from J_JLIM), an
  // actuator (LA_*), a joint-halves side (LS_* but LS_OWN; returns the body)
  auto img_joint = [&](auto&& put, int lane, int base, int j) {
    if (J == 0) return;
    const uint32_t* s = &B.w[H.o_joint + j * JOINT_STRIDE];
    const int bp = (int)s[J_BP], bc = (int)s[J_BC];
    const uint32_t* p = &B.w[H.o_body + bp * BODY_STRIDE];
    const uint32_t* c = &B.w[H.o_body + bc * BODY_STRIDE];
    const int ints[6] = {J_TYPE, J_BP, J_BC, J_FREE, J_ANGLE_OFF, J_NANGLES};
    for (int k = 0; k < 6; k++) put(lane, base + k, s[ints[k]]);
    put(lane, base + LJ_DAMP, s[J_DAMP]);
    put(lane, base + LJ_SP, s[J_SP]);
    put(lane, base + LJ_SA, s[J_SA]);
    for (int k = 0; k < 3; k++) {
      put(lane, base + LJ_OFFP + k, s[J_OFFP + k]);
      put(lane, base + LJ_OFFC + k, s[J_OFFC + k]);
      put(lane, base + LJ_IP + k, p[BODY_I + k]);
      put(lane, base + LJ_IC + k, c[BODY_I + k]);
    }
    for (int k = 0; k < 9; k++) {
      put(lane, base + LJ_AXP + k, s[J_AXP + k]);
      put(lane, base + LJ_AXC + k, s[J_AXC + k]);
    }
    for (int k = 0; k < 6; k++) put(lane, base + LJ_LIM + k, s[J_LIM + k]);
    put(lane, base + LJ_DOF, s[J_DOF]);
    put(lane, base + LJ_MP, p[BODY_MASS]);
    put(lane, base + LJ_MC, c[BODY_MASS]);
  };
  auto img_lim = [&](auto&& put, int lane, int base, int j, int row) {
    if (J == 0) return;
    const uint32_t* s = &B.w[H.o_joint + j * JOINT_STRIDE + J_JLIM + 8 * row];
    for (int k = 0; k < 6; k++) put(lane, base + k, s[k]);
  };
  auto img_act = [&](auto&& put, int lane, int base, int a) {
    if (K == 0) return;
    const uint32_t* s = &B.w[H.o_act + a * ACT_STRIDE];
    put(lane, base + LA_TYPE, s[A_TYPE]);
    put(lane, base + LA_JOINT, s[A_JOINT]);
    for (int k = 0; k < 3; k++) put(lane, base + LA_IDX + k, s[A_IDX + k]);
    put(lane, base + LA_STR, s[A_STR]);
  };
  auto img_side = [&](auto&& put, int lane, int base, int j, bool child) {
    const uint32_t* s = &B.w[H.o_joint + j * JOINT_STRIDE];
    const int body = (int)s[child ? J_BC : J_BP];
    const uint32_t* bw = &B.w[H.o_body + body * BODY_STRIDE];
    for (int k = 0; k < 3; k++) {
      put(lane, base + LS_OFF + k, s[(child ? J_OFFC : J_OFFP) + k]);
      put(lane, base + LS_AX0 + k, s[(child ? J_AXC : J_AXP) + k]);
      put(lane, base + LS_AX2 + k, s[(child ? J_AXC : J_AXP) + 6 + k]);
      put(lane, base + LS_I + k, bw[BODY_I + k]);
    }
    put(lane, base + LS_M, bw[BODY_MASS]);
    put(lane, base + LS_SG, fbits(child ? -1.0 : 1.0));
    put(lane, base + LS_BODY, (uint32_t)body);
    return body;
  };
  // the MULTI kernel's joint halves (MJ_*): revolute joints each driven by
  // the torque actuator of its index, <= 128 joints (16 lanes per 8)
  bool mjh = false;
  {
    bool ok = H.multi && J > 0 && J <= 128 && K == J && H.act_same;
    for (int j = 0; j < J; j++) ok = ok && d->joint_type[j] == BX_JOINT_REVOLUTE;
    for (int a = 0; a < K; a++) ok = ok && d->act_type[a] == BX_ACT_TORQUE;
    const bool off = getenv("BX_NO_MULTI_JH") && atoi(getenv("BX_NO_MULTI_JH"));
    mjh = ok && !off;
  }
  // MULTI threads per env: 128 when the bodies, joints (joint halves: two
  // lanes each), actuators and gather tasks (two per lane) fit, so four envs
  // share a CU (two waves each, 256 registers, <= 40 KB of LDS); else 256
  H.multi_L = (N <= 128 && K <= 128 && (mjh ? 2 * J <= 128 : J <= 128) && H.T <= 2 * 128 &&
               R <= 8 * 128) ? 128 : 256;
  if (mjh) {
    B.alloc((4 - (int)B.w.size() % 4) % 4);  // 16-byte aligned groups
    H.o_mjh = B.alloc(MJ_W * MJ_LANES);
    auto putm = [&](int lane, int w, uint32_t v) {
      B.w[H.o_mjh + (w / 4) * 4 * MJ_LANES + 4 * lane + w % 4] = v;
    };
    for (int l = 0; l < MJ_LANES; l++) {
      const int jx = (l >> 4) * 8 + (l & 7);
      const int j = jx < J ? jx : 0;
      img_joint(putm, l, MJ_JOINT, j);
      img_act(putm, l, MJ_ACT, j);
      img_lim(putm, l, MJ_JLIM, j, 0);
      img_side(putm, l, MJ_SIDE, j, (l & 8) != 0);
    }
  }
  if (H.single) {
    B.alloc((4 - (int)B.w.size() % 4) % 4);  // 16-byte aligned groups
    H.o_lane = B.alloc(LANE_W * LANE_IMG_LANES);
    auto put = [&](int lane, int w, uint32_t v) {
      B.w[H.o_lane + (w / 4) * 4 * LANE_IMG_LANES + 4 * lane + w % 4] = v;
    };
    auto put_joint = [&](int lane, int base, int j) { img_joint(put, lane, base, j); };
    auto put_lim = [&](int lane, int base, int j, int row) { img_lim(put, lane, base, j, row); };
    auto put_act = [&](int lane, int base, int a) { img_act(put, lane, base, a); };
    auto put_list = [&](int lane, int base, const std::vector<int>& v, bool has, uint32_t zero) {
      for (int k = 0; k < 8; k++) put(lane, base + k, has && k < (int)v.size() ? (uint32_t)v[k] : zero);
    };
    // a body's record: mass, inverse inertia, pos / rot / quat masks
    auto put_body = [&](int lane, int base, int b) {
      const uint32_t* s = &B.w[H.o_body + b * BODY_STRIDE];
      put(lane, base, s[BODY_MASS]);
      for (int k = 0; k < 3; k++) {
        put(lane, base + 1 + k, s[BODY_I + k]);
        put(lane, base + 4 + k, s[BODY_PM + k]);
        put(lane, base + 7 + k, s[BODY_RM + k]);
      }
      for (int k = 0; k < 4; k++) put(lane, base + 10 + k, s[BODY_QM + k]);
    };
    // joint halves: lane m's side body (the parent of joint m & 7 on lanes
    // 0-7 of each 16, the child on 8-15)
    auto side_body = [&](int m) {
      const int j = m & (HB - 1);
      const uint32_t* s = &B.w[H.o_joint + (j < J ? j : 0) * JOINT_STRIDE];
      return (int)s[(m & HB) ? J_BC : J_BP];
    };
    for (int l = 0; l < LANE_IMG_LANES; l++) {
      const bool hasB = l < N;
      const int b = hasB ? l : 0;
      put_body(l, LI_BODY, b);
      put_joint(l, LI_JOINT, l < J ? l : 0);
      put_act(l, LI_ACT, l < K ? l : 0);
      const int jh = l & (HB - 1);  // the lane's joint-halves joint
      put_joint(l, LI_JOINT_H, jh < J ? jh : 0);
      // the staged limit rows (stage_lim): lane l -> joint l
      put_lim(l, LI_JLIM, l < J ? l : 0, 0);
      put_lim(l, LI_JLIM12, l < J ? l : 0, 1);
      put_lim(l, LI_JLIM12 + 8, l < J ? l : 0, 2);
      put_lim(l, LI_JLIM_H, jh < J ? jh : 0, 0);
      if (J > 0) {
        // the joint-halves side: the parent's on lanes 0-7, the child's on
        // 8-15
        const bool child = (l & HB) != 0;
        const int body = img_side(put, l, LI_SIDE_H, jh < J ? jh : 0, child);
        // JB: the side body's record and gather lists; LS_OWN on the lowest
        // lane of the env's 16 whose side is that body
        const bool hasS = jh < J;
        bool own = hasS;
        for (int m = l & ~(2 * HB - 1); m < l; m++)
          if ((m & (HB - 1)) < J && side_body(m) == body) own = false;
        put(l, LI_SIDE_H + LS_OWN, own ? 1u : 0u);
        put_body(l, LI_BODY_J, body);
        put_list(l, LI_JL_J, jl[body], hasS, (uint32_t)(2 * J));
        put_list(l, LI_AL_J, al[body], hasS, (uint32_t)(2 * K));
        uint32_t czj = (uint32_t)(2 * R);
        if (hasS && !cl[body].empty()) czj |= (uint32_t)cl[body][0] & 0x7F000000u;
        put_list(l, LI_CL_J, cl[body], hasS, czj);
      }
      put_act(l, LI_ACT_H, jh < K ? jh : 0);
      if (R > 0) {
        uint32_t rw[32];
        row_words(l < R ? l : 0, rw);
        for (int k = 0; k < 32; k++) put(l, LI_ROW + k, rw[k]);
        // F_R2: the lane's two rows (slot1[l], slot2[l])
        if (r2 && l < 16) {
          const int a = slot1[l], b2 = slot2[l];
          row_words(a >= 0 ? a : 0, rw);
          for (int k = 0; k < 32; k++) put(l, LI_ROW + k, rw[k]);
          row_words(b2 >= 0 ? b2 : 0, rw);
          for (int k = 0; k < 32; k++) put(l, LI_ROW2 + k, rw[k]);
          put(l, LI_RIDX, (uint32_t)a);
          put(l, LI_RIDX + 1, (uint32_t)b2);
        }
      }
      put_list(l, LI_JL, jl[b], hasB, (uint32_t)(2 * J));
      put_list(l, LI_AL, al[b], hasB, (uint32_t)(2 * K));
      // contact entries carry their collider group in bits 24..30; the padding
      // entry takes the group of the body's first entry (it adds exact zeros)
      uint32_t cz = (uint32_t)(2 * R);
      if (hasB && !cl[b].empty()) cz |= (uint32_t)cl[b][0] & 0x7F000000u;
      put_list(l, LI_CL, cl[b], hasB, cz);
      // F_C16: entries 8..15 of the contact list
      for (int k = 0; k < 8; k++)
        put(l, LI_CL2 + k, hasB && 8 + k < (int)cl[b].size() ? (uint32_t)cl[b][8 + k] : cz);
    }
  }
  // the SINGLE kernel this system launches reads its joints' limit rows
  // from LDS when its feature set carries spherical joints (F_SPH; the
  // all-features instantiations too): carve the rows' region then (6
  // 16-byte groups per lane), not otherwise (Ant keeps its LDS footprint:
  // 32 envs per CU for the 2-wave kernels at 32,768 envs)
  if (H.single && (single_kernel_feat(L, system_feat(d, H, L, J, K, G, max_groups, xcol, jh_off, r2,
                                                     c16, r2g),
                                      (c16 ? mx_ja : mx) <= 4 ? 4 : 8) & 1)) {
    H.l_jlim = jlim_at;
    H.env_words = (jlim_at + 24 * L + 63) & ~63;
  }
  H.total_words = (int)B.w.size();
  std::memcpy(B.w.data(), &H, sizeof(BlobHdr));

  S->hdr = H;
  S->single_ok = H.single != 0;
  S->min_L = L;
  // gather width of the joint / actuator lists (and the contact list, unless
  // F_C16 gives it 16)
  S->gw = (c16 ? mx_ja : mx) <= 4 ? 4 : 8;
  {
    const int f = system_feat(d, H, L, J, K, G, max_groups, xcol, jh_off, r2, c16, r2g);
    S->feat = f;
    S->fold = (H.act_same && K == J && J > 0 && !(f & 2)) ? 1 : 0;
    // JB (the Ant / HalfCheetah env kernels: joint halves own body copies):
    // JB's body conditions (jb_bodies_ok) and no forces (they index bodies
    // by lane)
    // (BX_NO_JB=1: off, the Ant / HalfCheetah kinds then take the all-kinds
    // kernel; the GPU tests run that fallback against the goldens too)
    const bool jb_off = getenv("BX_NO_JB") && atoi(getenv("BX_NO_JB"));
    const bool jb = S->fold && (f & 128) && !(f & 16) && L == 16 && !jb_off && jb_bodies_ok();
    S->jb = jb ? 1 : 0;
  }
  // the MULTI kernel is instantiated for the lean feature set (revolute,
  // torque, capsule-plane / capsule-capsule, no forces)
  S->multi_ok = H.multi != 0 && (S->feat & (1 | 2 | 16 | 64)) == 0;
  S->mode = S->single_ok ? 1 : (S->multi_ok ? 3 : 0);
  S->host = std::move(B.w);
  S->L = S->multi_ok ? H.multi_L : L;
  S->tpb = S->L > 64 ? S->L : 64;
  S->lds_env = (size_t)(L > 64 ? 1 : 64 / L) * H.env_words * 4;
  S->lds_reset = (size_t)64 * N * 13 * 4;
  if (S->lds_env > 160 * 1024) return fail("system too large for one workgroup's LDS");
  if (r && S->lds_reset > 160 * 1024) return fail("system too large for the reset kernel's LDS");
  return 0;
}

hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

// Every entry point that touches device memory runs with the system's device
// current and restores the caller's afterwards (HIP launches go to the current
// device; a process may hold systems on several GPUs).
struct DeviceScope {
  int prev = -1, want;
  hipError_t err = hipSuccess;
  explicit DeviceScope(int d) : want(d) {
    err = hipGetDevice(&prev);
    if (err == hipSuccess && prev != want) err = hipSetDevice(want);
  }
  ~DeviceScope() {
    if (prev >= 0 && prev != want) (void)hipSetDevice(prev);
  }
};
#define DEVICE_SCOPE(S)                                                             \
  DeviceScope _dev((S)->device);                                                    \
  if (_dev.err != hipSuccess) return fail(std::string("device ") + std::to_string((S)->device) + \
                                          ": " + hipGetErrorString(_dev.err))

// obs / metric widths of each env kind's layer (the kernel's obs_elem and
// reward code), from the system's shape: ant.py:257-282, humanoid.py:282-334,
// half_cheetah.py:200-214, humanoid_standup.py:249-289
int env_sizes(const bx_system* S, const bx_env_params* P, int* obs, int* met) {
  const BlobHdr& H = S->hdr;
  const int D = H.D, N = H.N;
  const bool xy = (P->obs_flags & BX_OBS_XY) != 0;
  if (P->obs_flags & ~BX_OBS_XY) return fail("unknown obs_flags bits");
  switch (P->kind) {
    case BX_ENV_ANT:
      *obs = 1 + 4 + D + 3 + 3 + D + (P->coef[7] != 0.f ? 6 * N : 0) + (xy ? 2 : 0);
      *met = 10;
      return 0;
    case BX_ENV_HUMANOID:
    case BX_ENV_HUMANOID_STANDUP: {
      if (xy && P->kind == BX_ENV_HUMANOID_STANDUP)
        return fail("HumanoidStandup has no current-position observation option");
      int qfrc = 0;
      for (int a = 0; a < H.K; a++) {
        int j = (int)S->host[H.o_act + a * ACT_STRIDE + A_JOINT];
        qfrc += (int)S->host[H.o_joint + j * JOINT_STRIDE + J_DOF];
      }
      *obs = 1 + 4 + D + 3 + 3 + D + 15 * (N - 1) + qfrc + (xy ? 2 : 0);
      *met = P->kind == BX_ENV_HUMANOID ? 9 : 2;
      return 0;
    }
    case BX_ENV_HOPPER:
    case BX_ENV_WALKER2D:
      // (x,) z, ang_y, joint angles, vel x, vel z, ang y, joint vels (hopper.py:231-246)
      *obs = (xy ? 2 : 1) + 1 + D + 3 + D;
      *met = 5;
      return 0;
    case BX_ENV_INVERTED_PENDULUM:  // cart x, joint angles, cart vel x, joint vels
      if (xy) return fail("this env has no current-position observation option");
      *obs = 2 + 2 * D;
      *met = 0;
      return 0;
    case BX_ENV_INVERTED_DOUBLE_PENDULUM:  // cart x, sin, cos, cart vel x, joint vels
      if (xy) return fail("this env has no current-position observation option");
      *obs = 2 + 3 * D;
      *met = 0;
      return 0;
    case BX_ENV_ACROBOT:  // joint angles, joint vels
      if (xy) return fail("this env has no current-position observation option");
      *obs = 2 * D;
      *met = 4;
      return 0;
    case BX_ENV_REACHER:
    case BX_ENV_REACHERANGLE:  // cos, sin, target xy, tip vel xy, tip - target
      if (xy) return fail("this env has no current-position observation option");
      if (P->kind == BX_ENV_REACHERANGLE && H.A > 2)
        return fail("ReacherAngle's action map holds at most 2 actions");
      *obs = 2 * D + 7;
      *met = 2;
      return 0;
    case BX_ENV_SWIMMER:  // (x, y,) ang z, joint angles, vel x, vel y, ang z, joint vels
      if (N != 4) return fail("Swimmer's drag program takes 3 segments and a floor");
      *obs = (xy ? 3 : 1) + D + 3 + D;
      *met = 8;
      return 0;
    case BX_ENV_PUSHER:  // joint angles, joint vels, tip, object, goal positions
      if (xy) return fail("this env has no current-position observation option");
      *obs = 2 * D + 9;
      *met = 3;
      return 0;
    case BX_ENV_UR5E:
    case BX_ENV_FETCH:  // fwd, up, |target|, target dir, local pos, local vel, contacts
      if (xy) return fail("this env has no current-position observation option");
      *obs = 10 + 7 * N;
      *met = P->kind == BX_ENV_UR5E ? 3 : 5;
      return 0;
    case BX_ENV_GRASP:  // object, target, local pos / vel, hand and object terms, contacts
      if (xy) return fail("this env has no current-position observation option");
      if (N < 16) return fail("Grasp's reward reads the contacts of bodies 3, 9, 12 and 15");
      *obs = 1 + 3 + 1 + 3 + 6 * N + 3 + 3 + 1 + 1 + 3 + 1 + N;
      *met = 5;
      return 0;
    case BX_ENV_HALFCHEETAH:
      *obs = 3 + D + 3 + D + (xy ? 1 : 0);
      *met = 4;
      return 0;
  }
  return fail("unknown env kind");
}

int check_env(const bx_system* S, const bx_env_params* P) {
  int obs = 0, met = 0;
  if (env_sizes(S, P, &obs, &met)) return 1;
  if (P->obs_size != obs)
    return fail("obs_size " + std::to_string(P->obs_size) + " != " + std::to_string(obs) +
                " for this env kind and system");
  if (P->n_metrics != met)
    return fail("n_metrics " + std::to_string(P->n_metrics) + " != " + std::to_string(met) +
                " for this env kind");
  return 0;
}

size_t step_lds(const bx_system* S) {
  if (S->mode == 3) return (size_t)S->hdr.env_words_m * 4;
  size_t b = (size_t)(S->tpb / S->L) * S->hdr.env_words * 4;
  if (S->mode == 2) b += (size_t)S->hdr.const_words * 4;
  return b;
}

bool field_ok(const bx_field& f) { return f.ptr != nullptr; }
bool qp_ok(const bx_qp& q) {
  return field_ok(q.pos) && field_ok(q.rot) && field_ok(q.vel) && field_ok(q.ang);
}

}  // namespace

extern "C" {

int bx_abi_version(void) { return BX_ABI_VERSION; }

const char* bx_last_error(void) { return g_err.c_str(); }

int bx_device_count(int* count) {
  HIP_OK(hipGetDeviceCount(count));
  return 0;
}

int bx_system_create(const bx_desc* desc, const bx_reset_desc* reset, int device, bx_system** out) {
  if (!desc || !out) return fail("null argument");
  bx_system* S = new bx_system();
  S->device = device;
  if (int rc = build_blob(desc, reset, S)) {
    delete S;
    return rc;
  }
  DeviceScope dev(device);
  hipError_t e = dev.err;
  if (e == hipSuccess) e = hipMalloc(&S->blob, S->host.size() * 4);
  if (e == hipSuccess) e = hipMemcpy(S->blob, S->host.data(), S->host.size() * 4, hipMemcpyHostToDevice);
  if (e != hipSuccess) {
    std::string m = std::string("device setup: ") + hipGetErrorString(e);
    if (S->blob) (void)hipFree(S->blob);
    delete S;
    return fail(m);
  }
  *out = S;
  return 0;
}

int bx_system_destroy(bx_system* S) {
  if (!S) return 0;
  if (S->blob || S->movf) {
    DEVICE_SCOPE(S);
    if (S->movf) HIP_OK(hipFree(S->movf));
    if (S->blob) HIP_OK(hipFree(S->blob));
  }
  delete S;
  return 0;
}

// the host half of bx_system_create: the kernel plan of a descriptor (no device)
int bx_system_plan(const bx_desc* desc, const bx_reset_desc* reset, int32_t* mode,
                   int32_t* lanes, int32_t* lds_bytes) {
  if (!desc || !mode || !lanes || !lds_bytes) return fail("null argument");
  bx_system S;
  if (int rc = build_blob(desc, reset, &S)) return rc;
  *mode = S.mode;
  *lanes = S.L;
  *lds_bytes = (int32_t)step_lds(&S);
  return 0;
}

int bx_system_lanes(bx_system* S) { return S ? S->L : 0; }
int bx_system_env_lanes(bx_system* S) {
  return S ? S->L : 0;
}
int bx_system_lds_bytes(bx_system* S) { return S ? (int)step_lds(S) : 0; }

int bx_system_set_single(bx_system* S, int on) {
  if (!S) return fail("null system");
  if (on && (!S->single_ok || S->L != S->min_L)) return fail("system does not fit the single-item-per-lane kernel");
  S->mode = on ? 1 : 0;
  return 0;
}

int bx_system_set_variant(bx_system* S, int lanes, int mode) {
  if (!S) return fail("null system");
  if (lanes != 16 && lanes != 32 && lanes != 64 && lanes != 128 && lanes != 256)
    return fail("lanes must be 16, 32, 64, 128 or 256");
  if (mode < 0 || mode > 3) return fail("mode must be 0 (global), 1 (single), 2 (lds) or 3 (multi)");
  if (mode == 1 && (!S->single_ok || lanes < S->min_L || lanes > 64 || lanes > S->hdr.L))
    return fail("system does not fit the single-item-per-lane kernel at that width");
  if (mode == 3 && (!S->multi_ok || (lanes != 256 && !(lanes == 128 && S->hdr.multi_L == 128))))
    return fail("system does not fit the MULTI-mode kernel at that width (128 or 256 lanes)");
  int old_L = S->L, old_m = S->mode, old_t = S->tpb;
  S->L = lanes;
  S->mode = mode;
  if (lanes > 64) S->tpb = lanes;
  else if (S->tpb > 64 || S->tpb % lanes) S->tpb = 64;
  if (step_lds(S) > 160 * 1024) {
    S->L = old_L;
    S->mode = old_m;
    S->tpb = old_t;
    return fail("variant exceeds the LDS budget");
  }
  return 0;
}

int bx_system_set_block(bx_system* S, int threads) {
  if (!S) return fail("null system");
  if (threads < S->L || threads > (S->L > 64 ? S->L : 64) || threads % S->L)
    return fail("threads must be a multiple of the lanes per env, at most 64 (or the lanes "
                "per env past 64)");
  int old = S->tpb;
  S->tpb = threads;
  if (step_lds(S) > 160 * 1024) {
    S->tpb = old;
    return fail("block exceeds the LDS budget");
  }
  return 0;
}

// the step reads actions through jp.take-style clipped indices (jumpy.py:151):
// any positive width is valid, 0 only when the system reads no action
static int check_act(const bx_system* S, const float* act, int64_t act_stride, int64_t act_width) {
  const bool reads = S->hdr.K > 0 || S->hdr.NF > 0;
  if (act_width < 0 || act_stride < 0) return fail("negative action width or stride");
  if (reads && (!act || act_width == 0)) return fail("null or empty action");
  return 0;
}

int bx_system_step(bx_system* S, int64_t n_envs, const bx_qp* qin, const float* act,
                   int64_t act_stride, int64_t act_width, const bx_qp* qout, const bx_info* info,
                   void* stream) {
  if (!S || !qin || !qout) return fail("null argument");
  DEVICE_SCOPE(S);
  if (n_envs <= 0) return n_envs == 0 ? 0 : fail("negative n_envs");
  if (!qp_ok(*qin) || !qp_ok(*qout)) return fail("null qp field");
  if (check_act(S, act, act_stride, act_width)) return 1;
  StepArgs a{};
  a.blob = S->blob;
  a.n_envs = n_envs;
  a.qin = *qin;
  a.qout = *qout;
  a.act = act;
  a.act_stride = act_stride;
  a.act_width = act_width;
  if (info) a.info = *info;
  if (S->mode == 3 && S->hdr.R > MCBUF && S->movf_envs < n_envs) {
    // the overflow contacts (a pass with more than MCBUF penetrating rows):
    // grown to this batch once; a capture cannot allocate
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    HIP_OK(hipStreamIsCapturing(as_stream(stream), &cs));
    if (cs != hipStreamCaptureStatusNone)
      return fail("MULTI overflow buffer: step the batch once before capturing it");
    HIP_OK(hipStreamSynchronize(as_stream(stream)));
    if (S->movf) HIP_OK(hipFree(S->movf));
    S->movf = nullptr;
    S->movf_envs = 0;
    HIP_OK(hipMalloc(&S->movf, (size_t)n_envs * (S->hdr.R - MCBUF) * MOVF_W * 4));
    S->movf_envs = n_envs;
  }
  a.movf = S->movf;
  if (S->mode == 1)
    HIP_OK(launch_system_step_single(S->L, S->feat, S->gw, S->tpb, n_envs, step_lds(S), as_stream(stream), a));
  else if (S->mode == 3)
    HIP_OK(launch_system_step_multi(S->L, S->hdr.o_mjh ? 1 : 0, n_envs, step_lds(S), as_stream(stream), a));
  else
    HIP_OK(launch_system_step_generic(S->L, S->mode, S->feat, S->tpb, n_envs, step_lds(S), as_stream(stream), a));
  return 0;
}

// bx_env_step over n_steps consecutive steps in one launch (bx_env_rollout_packed):
// step t reads act + t * act_step and writes the out pointers + t * out_step
struct DrawSpec {  // bx_env_rollout_random's on-device action draws
  uint64_t seed, offset, step;
  float lo, hi;
  float* act_out;
};
static int check_draw(const bx_system* S, const bx_env_params* env, int64_t act_width) {
  if (act_width <= 0) return fail("on-device draws need act_width >= 1");
  // env programs that read the raw action row themselves (the pre-step
  // action maps, the humanoid qfrc observation)
  const int k = env->kind;
  if (k == BX_ENV_REACHERANGLE || k == BX_ENV_SWIMMER || k == BX_ENV_GRASP ||
      k == BX_ENV_HUMANOID || k == BX_ENV_HUMANOID_STANDUP)
    return fail("this env kind's program reads the action row itself: draw with bx_uniform_slabs");
  if (act_width > S->hdr.act_read)
    return fail("on-device draws stage the whole action row: act_width exceeds the row the system stages");
  return 0;
}

static int env_step_impl(bx_system* S, const bx_env_params* env, int64_t n_envs,
                         const bx_env_state* in, const float* act, int64_t act_stride,
                         int64_t act_width, const bx_env_state* out, void* stream,
                         int32_t n_steps, int64_t act_step, int64_t out_step, int64_t rng_step,
                         const DrawSpec* draw = nullptr, bool packed = false) {
  if (!S || !env || !in || !out) return fail("null argument");
  DEVICE_SCOPE(S);
  if (check_env(S, env)) return 1;
  // an empty batch is a no-op (its buffers, the action included, may be null)
  if (n_envs <= 0) return n_envs == 0 ? 0 : fail("negative n_envs");
  if (draw ? check_draw(S, env, act_width) : check_act(S, act, act_stride, act_width)) return 1;
  if (!qp_ok(in->qp) || !qp_ok(out->qp)) return fail("null qp field");
  if (!in->done || !out->done || !out->reward || !out->obs) return fail("null env buffer");
  if (env->auto_reset && (!qp_ok(env->first_qp) || !env->first_obs))
    return fail("auto_reset needs first_qp and first_obs");
  if (env->kind == BX_ENV_GRASP && !env->act_map) return fail("Grasp needs its action map");
  if (env->kind == BX_ENV_GRASP && act_width + 0 > S->hdr.xact_words)
    return fail("action wider than the env program's action buffer");
  if ((env->kind == BX_ENV_UR5E || env->kind == BX_ENV_FETCH || env->kind == BX_ENV_GRASP) &&
      (!in->rng || !out->rng))
    return fail("the target envs need the per-env rng stream (in and out)");
  if (env->episode_length > 0 && (!out->steps || !out->truncation))
    return fail("episode wrapper needs steps and truncation buffers");
  EnvArgs a{};
  a.blob = S->blob;
  a.lane_img = S->blob + S->hdr.o_lane;
  a.hdr = S->hdr;
  a.n_envs = n_envs;
  a.P = *env;
  a.in = *in;
  a.out = *out;
  a.act = act;
  a.act_stride = act_stride;
  a.act_width = act_width;
  a.n_steps = n_steps;
  a.act_step = act_step;
  a.out_step = out_step;
  a.rng_step = rng_step;
  a.packed = packed ? 1 : 0;
  if (draw) {
    a.draw = 1;
    a.draw_seed = draw->seed;
    a.draw_offset = draw->offset;
    a.draw_step = draw->step;
    a.draw_lo = draw->lo;
    a.draw_hi = draw->hi;
    a.act_out = draw->act_out;
  }
  if (S->mode == 1)
    HIP_OK(launch_env_step_single(S->L, S->feat, S->gw, S->tpb, n_envs, step_lds(S), as_stream(stream), a,
                                  S->fold ? (1 | (S->jb ? 2 : 0)) : 0));
  else if (S->mode == 3)  // MULTI-mode systems step envs with the item-loop kernel
    HIP_OK(launch_env_step_generic(S->L, 0, S->feat, S->tpb, n_envs,
                                   (size_t)S->hdr.env_words * 4, as_stream(stream), a));
  else
    HIP_OK(launch_env_step_generic(S->L, S->mode, S->feat, S->tpb, n_envs, step_lds(S), as_stream(stream), a));
  return 0;
}

int bx_env_step(bx_system* S, const bx_env_params* env, int64_t n_envs, const bx_env_state* in,
                const float* act, int64_t act_stride, int64_t act_width, const bx_env_state* out,
                void* stream) {
  return env_step_impl(S, env, n_envs, in, act, act_stride, act_width, out, stream, 1, 0, 0, 0);
}

static int env_step_packed(bx_system* S, const bx_env_params* env, int64_t n_envs, int32_t n_steps,
                           const float* qp_in, const float* done_in, const float* steps_in,
                           const uint32_t* rng_in, const float* act, int64_t act_stride,
                           int64_t act_step, int64_t act_width, float* out, uint32_t* rng_out,
                           void* stream, const DrawSpec* draw = nullptr) {
  if (!S || !env) return fail("null argument");
  if (n_envs <= 0) {
    if (check_env(S, env)) return 1;
    return n_envs == 0 ? 0 : fail("negative n_envs");
  }
  if (!qp_in || !out) return fail("null argument");
  const int64_t N = S->hdr.N, B = n_envs;
  auto packed = [&](float* base) {
    bx_qp q;
    const int64_t es = N * 16;
    q.pos = bx_field{base, es, 16};
    q.rot = bx_field{base + 3, es, 16};
    q.vel = bx_field{base + 7, es, 16};
    q.ang = bx_field{base + 10, es, 16};
    return q;
  };
  bx_env_state in{};
  in.qp = packed(const_cast<float*>(qp_in));
  in.done = const_cast<float*>(done_in);
  in.steps = const_cast<float*>(steps_in);
  in.rng = const_cast<uint32_t*>(rng_in);
  bx_env_state o{};
  o.qp = packed(out);
  float* p = out + B * N * 16;
  o.obs = p;
  p += B * env->obs_size;
  o.reward = p;
  o.done = p + B;
  o.steps = p + 2 * B;
  o.truncation = p + 3 * B;
  o.metrics = env->n_metrics > 0 ? p + 4 * B : nullptr;
  o.rng = rng_out;
  // one step's output block: qp | obs | reward, done, steps, truncation | metrics
  const int64_t block = B * (N * 16 + env->obs_size + 4 + env->n_metrics);
  return env_step_impl(S, env, n_envs, &in, act, act_stride, act_width, &o, stream, n_steps,
                       act_step, block, B, draw, true);
}

int bx_env_step_packed(bx_system* S, const bx_env_params* env, int64_t n_envs,
                       const float* qp_in, const float* done_in, const float* steps_in,
                       const uint32_t* rng_in, const float* act, int64_t act_stride,
                       int64_t act_width, float* out, uint32_t* rng_out, void* stream) {
  return env_step_packed(S, env, n_envs, 1, qp_in, done_in, steps_in, rng_in, act, act_stride, 0,
                         act_width, out, rng_out, stream);
}

int bx_env_rollout_packed(bx_system* S, const bx_env_params* env, int64_t n_envs, int32_t n_steps,
                          const float* qp_in, const float* done_in, const float* steps_in,
                          const uint32_t* rng_in, const float* act, int64_t act_stride,
                          int64_t act_step_stride, int64_t act_width, float* out,
                          uint32_t* rng_out, void* stream) {
  if (n_steps < 0) return fail("negative n_steps");
  if (n_steps == 0) return S && env ? check_env(S, env) : fail("null argument");
  if (act_step_stride < 0) return fail("negative action step stride");
  return env_step_packed(S, env, n_envs, n_steps, qp_in, done_in, steps_in, rng_in, act,
                         act_stride, act_step_stride, act_width, out, rng_out, stream);
}

int bx_env_rollout_random(bx_system* S, const bx_env_params* env, int64_t n_envs, int32_t n_steps,
                          const float* qp_in, const float* done_in, const float* steps_in,
                          const uint32_t* rng_in, uint64_t seed, uint64_t offset,
                          uint64_t step_stride, float lo, float hi, int64_t act_width,
                          float* act_out, float* out, uint32_t* rng_out, void* stream) {
  if (!S || !env) return fail("null argument");
  if (n_steps < 0) return fail("negative n_steps");
  if (check_env(S, env) || check_draw(S, env, act_width)) return 1;
  if (n_steps == 0) return 0;
  const DrawSpec d{seed, offset, step_stride, lo, hi, act_out};
  return env_step_packed(S, env, n_envs, n_steps, qp_in, done_in, steps_in, rng_in, nullptr, 0, 0,
                         act_width, out, rng_out, stream, &d);
}

int bx_system_info(bx_system* S, int64_t n_envs, const bx_qp* qp, const bx_info* info, void* stream) {
  if (!S || !qp || !info) return fail("null argument");
  DEVICE_SCOPE(S);
  if (n_envs <= 0) return n_envs == 0 ? 0 : fail("negative n_envs");
  InfoArgs a{};
  a.blob = S->blob;
  a.n_envs = n_envs;
  a.q = *qp;
  a.info = *info;
  HIP_OK(launch_info_obs(S->L, n_envs, S->lds_env, as_stream(stream), a));
  return 0;
}

int bx_env_observe(bx_system* S, const bx_env_params* env, int64_t n_envs, const bx_qp* qp,
                   const float* act, int64_t act_stride, int64_t act_width, float* obs,
                   void* stream) {
  if (!S || !env || !qp || !obs) return fail("null argument");
  DEVICE_SCOPE(S);
  if (check_env(S, env)) return 1;
  if (act_width < 0 || act_stride < 0) return fail("negative action width or stride");
  if ((env->kind == BX_ENV_HUMANOID || env->kind == BX_ENV_HUMANOID_STANDUP) && S->hdr.K > 0 &&
      (!act || act_width == 0))
    return fail("the humanoid observation reads the action (qfrc_actuator)");
  if (n_envs <= 0) return n_envs == 0 ? 0 : fail("negative n_envs");
  InfoArgs a{};
  a.blob = S->blob;
  a.n_envs = n_envs;
  a.q = *qp;
  a.kind = env->kind;
  a.obs_size = env->obs_size;
  a.obs_flags = env->obs_flags;
  for (int k = 0; k < 8; k++) a.coef[k] = env->coef[k];
  a.act = act;
  a.act_stride = act_stride;
  a.act_width = act_width;
  a.obs = obs;
  HIP_OK(launch_info_obs(S->L, n_envs, S->lds_env, as_stream(stream), a));
  return 0;
}

int bx_system_joint_angles(bx_system* S, int64_t n_envs, const bx_qp* qp, float* angle,
                           float* vel, void* stream) {
  if (!S || !qp) return fail("null argument");
  DEVICE_SCOPE(S);
  if (n_envs <= 0) return n_envs == 0 ? 0 : fail("negative n_envs");
  if (S->hdr.D == 0) return 0;
  if (!angle || !vel) return fail("null angle or velocity buffer");
  InfoArgs a{};
  a.blob = S->blob;
  a.n_envs = n_envs;
  a.q = *qp;
  a.angle = angle;
  a.angvel = vel;
  HIP_OK(launch_info_obs(S->L, n_envs, S->lds_env, as_stream(stream), a));
  return 0;
}

int bx_env_sizes(bx_system* S, const bx_env_params* env, int32_t* obs_size, int32_t* n_metrics) {
  if (!S || !env || !obs_size || !n_metrics) return fail("null argument");
  int o = 0, m = 0;
  if (env_sizes(S, env, &o, &m)) return 1;
  *obs_size = o;
  *n_metrics = m;
  return 0;
}

int bx_env_reset(bx_system* S, const bx_env_params* env, int64_t n_envs, uint64_t seed,
                 int64_t env_offset, const uint64_t* env_seeds, float noise_scale,
                 const bx_env_state* out, void* stream) {
  if (!S || !env || !out) return fail("null argument");
  DEVICE_SCOPE(S);
  if (S->hdr.o_base == 0) return fail("system was created without a reset descriptor");
  if (check_env(S, env)) return 1;
  if (n_envs <= 0) return n_envs == 0 ? 0 : fail("negative n_envs");
  if (env_offset < 0) return fail("negative env_offset");
  if (!(noise_scale >= 0.f)) return fail("noise_scale must be >= 0");
  if (!qp_ok(out->qp) || !out->obs || !out->reward || !out->done) return fail("null env buffer");
  if (env->n_metrics > 0 && !out->metrics) return fail("null metrics buffer");
  ResetArgs r{};
  r.blob = S->blob;
  r.n_envs = n_envs;
  r.out = out->qp;
  r.gen = 1;
  r.seed = seed;
  r.env_offset = env_offset;
  r.seeds = env_seeds;
  r.scale = noise_scale;
  r.kind = env->kind;
  for (int k = 0; k < 8; k++) r.coef[k] = env->coef[k];
  r.rng_out = out->rng;
  // the bodies a reset program places must exist (coef holds their indices)
  auto body_ok = [&](float x) { return x >= 0.f && x < (float)S->hdr.N && x == (float)(int)x; };
  if ((env->kind == BX_ENV_REACHER || env->kind == BX_ENV_REACHERANGLE) && !body_ok(env->coef[0]))
    return fail("reacher reset: coef[0] must be the target body");
  if (env->kind == BX_ENV_PUSHER &&
      !(body_ok(env->coef[1]) && body_ok(env->coef[2]) && body_ok(env->coef[3])))
    return fail("pusher reset: coef[1..3] must be the object, goal and table bodies");
  if (env->kind == BX_ENV_PUSHER && S->hdr.num_joint_dof < 4)
    return fail("pusher reset: the last 4 dofs get no velocity noise; the system has fewer");
  if ((env->kind == BX_ENV_UR5E || env->kind == BX_ENV_FETCH) && !body_ok(env->coef[1]))
    return fail("target env reset: coef[1] must be the target body");
  if ((env->kind == BX_ENV_UR5E || env->kind == BX_ENV_FETCH || env->kind == BX_ENV_GRASP) &&
      !out->rng)
    return fail("the target envs' reset writes their per-env rng stream: out->rng is null");
  HIP_OK(launch_default_qp(n_envs, S->lds_reset, as_stream(stream), r));
  InfoArgs a{};
  a.blob = S->blob;
  a.n_envs = n_envs;
  a.q = out->qp;
  a.kind = env->kind;
  a.obs_size = env->obs_size;
  a.obs_flags = env->obs_flags;
  for (int k = 0; k < 8; k++) a.coef[k] = env->coef[k];
  a.obs = out->obs;
  // _get_obs(qp, info, jp.zeros(action_size)): a null action reads as zeros
  a.act = nullptr;
  a.act_width = 0;
  a.zero_reward = out->reward;
  a.zero_done = out->done;
  a.zero_steps = out->steps;
  a.zero_trunc = out->truncation;
  a.zero_metrics = out->metrics;
  a.n_metrics = env->n_metrics;
  HIP_OK(launch_info_obs(S->L, n_envs, S->lds_env, as_stream(stream), a));
  return 0;
}

int bx_system_default_qp(bx_system* S, int64_t n_envs, const float* joint_angle,
                         const float* joint_velocity, const bx_qp* qp_out, void* stream) {
  if (!S || !qp_out) return fail("null argument");
  DEVICE_SCOPE(S);
  if (S->hdr.o_base == 0) return fail("system was created without a reset descriptor");
  if (n_envs <= 0) return n_envs == 0 ? 0 : fail("negative n_envs");
  if (S->hdr.num_joint_dof > 0 && (!joint_angle || !joint_velocity)) return fail("null joint arrays");
  ResetArgs a{};
  a.blob = S->blob;
  a.n_envs = n_envs;
  a.angle = joint_angle;
  a.vel = joint_velocity;
  a.out = *qp_out;
  HIP_OK(launch_default_qp(n_envs, S->lds_reset, as_stream(stream), a));
  return 0;
}

static bool aligned16(const void* p) { return ((uintptr_t)p & 15) == 0; }

int bx_phase(bx_system* S, int which, int64_t n_envs, int64_t plane, const float* in, float* out,
             const float* aux, int64_t aux_plane, void* stream) {
  if (!S || !in || !out) return fail("null argument");
  DEVICE_SCOPE(S);
  if (which < 0 || which > 2) return fail("unknown phase");
  if (n_envs <= 0 || n_envs % 4) return fail("n_envs must be a positive multiple of 4");
  const int64_t N = S->hdr.N;
  if (N * n_envs >= (int64_t)1 << 32) return fail("too many bodies for one phase launch");
  if (plane < N * n_envs || plane % 4) return fail("plane stride must be >= N*n_envs and a multiple of 4");
  if (which >= 1 && (!aux || aux_plane % 4 || aux_plane < N * n_envs)) return fail("bad aux planes");
  if (!aligned16(in) || !aligned16(out) || (aux && !aligned16(aux))) return fail("SoA bases must be 16-byte aligned");
  HIP_OK(launch_phase(which, S->blob, (int)N, n_envs, plane, in, out, aux, aux_plane, as_stream(stream)));
  return 0;
}

int bx_phase_capsule_plane(bx_system* S, int64_t n_envs, int64_t plane, const float* in, float* out,
                           int64_t out_plane, void* stream) {
  if (!S || !in || !out) return fail("null argument");
  DEVICE_SCOPE(S);
  if (n_envs <= 0 || n_envs % 4) return fail("n_envs must be a positive multiple of 4");
  const int64_t N = S->hdr.N, R = S->hdr.R;
  if (plane < N * n_envs || plane % 4) return fail("plane stride must be >= N*n_envs and a multiple of 4");
  if (out_plane < R * n_envs || out_plane % 4) return fail("out plane stride must be >= R*n_envs");
  if (!aligned16(in) || !aligned16(out)) return fail("SoA bases must be 16-byte aligned");
  if (R == 0) return 0;
  HIP_OK(launch_capsule_plane(S->blob, (int)R, n_envs, plane, in, out, out_plane, as_stream(stream)));
  return 0;
}

int bx_debug_partner(float* out64, int lanes, void* stream) {
  if (!out64) return fail("null argument");
  if (lanes != 16) return fail("lanes must be 16 (the revolute joint halves' exchange)");
  HIP_OK(debug_partner(out64, lanes, as_stream(stream)));
  return 0;
}

int bx_debug_stamps(unsigned long long* out, int reset) {
  // bit 1 of reset selects the MULTI-mode stamps (BX_MSTAMPS build)
  // bit 2: the per-workgroup sums (4096 x 16 entries) instead of the totals
  if (reset & 2) HIP_OK(debug_mstamps(out, reset & 1));
  else HIP_OK(debug_stamps(out, reset));
  return 0;
}

int bx_uniform(float* out, int64_t n, uint64_t seed, uint64_t offset, float lo, float hi, void* stream) {
  return bx_uniform_slabs(out, n, 1, seed, offset, 0, nullptr, 0, lo, hi, stream);
}

int bx_uniform_epoch(float* out, int64_t n, uint64_t seed, uint64_t offset, const int64_t* epoch,
                     uint64_t epoch_stride, float lo, float hi, void* stream) {
  if (!epoch && n > 0) return fail("null epoch counter");
  return bx_uniform_slabs(out, n, 1, seed, offset, 0, epoch, epoch_stride, lo, hi, stream);
}

int bx_uniform_slabs(float* out, int64_t slab_n, int64_t n_slabs, uint64_t seed, uint64_t offset,
                     uint64_t slab_stride, const int64_t* epoch, uint64_t epoch_stride, float lo,
                     float hi, void* stream) {
  if (slab_n < 0 || n_slabs < 0) return fail("negative size");
  if (slab_n == 0 || n_slabs == 0) return 0;
  if (slab_n > INT64_MAX / n_slabs || slab_n * n_slabs > ((int64_t)1 << 40))
    return fail("too many elements for one draw");
  if (!out) return fail("null output");
  // no system handle here: launch on the device that owns the stream (the
  // caller's current device for the null stream)
  int dev = -1;
  hipStream_t st = as_stream(stream);
  if (st) HIP_OK(hipStreamGetDevice(st, &dev));
  else HIP_OK(hipGetDevice(&dev));
  DeviceScope scope(dev);
  if (scope.err != hipSuccess) return fail(std::string("device: ") + hipGetErrorString(scope.err));
  HIP_OK(launch_uniform_slabs(out, slab_n, n_slabs, seed, offset, slab_stride, epoch, epoch_stride,
                              lo, hi, st));
  return 0;
}

}  // extern "C"
