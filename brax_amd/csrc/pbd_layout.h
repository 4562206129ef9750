// pbd_layout.h — device constant-blob and per-env LDS layout (host + device).
//
// The blob is one read-only array of 32-bit words in HBM (floats bit-cast):
// a BlobHdr followed by fixed-stride records for bodies, joints, actuators,
// contact rows, the per-body gather lists that replace the reference's
// `segment_sum`s, and the reset (forward-kinematics) tables.
#pragma once
#include <stdint.h>

#include "../../include/brax_amd.h"

namespace bx {

// record strides (words) and field offsets
enum {
  BODY_STRIDE = 16,
  BODY_MASS = 0, BODY_I = 2, BODY_PM = 5, BODY_RM = 8, BODY_QM = 11,
};
enum {
  JOINT_STRIDE = 72,
  J_TYPE = 0, J_BP = 1, J_BC = 2, J_FREE = 3, J_DOF = 4, J_ANGLE_OFF = 5, J_NANGLES = 6,
  J_DAMP = 7, J_SP = 8, J_SA = 9, J_OFFP = 10, J_OFFC = 13, J_AXP = 16, J_AXC = 25, J_LIM = 34,
  // legacy_spring joints (spring_joints.py:57-67)
  J_STIFF = 40, J_SDAMP = 41, J_LSTR = 42,
  // the three limit rows as the kernels test them (LL_*, 8 words each): the
  // item-loop kernels' atan2-free hinge and limit rows read them here, the
  // SINGLE kernels from the lane image (LI_JLIM, LI_JLIM12)
  J_JLIM = 48,
};
enum { ACT_STRIDE = 8, A_TYPE = 0, A_JOINT = 1, A_IDX = 2, A_STR = 5 };
// collider groups: NearNeighbors cutoff (0 = Pairs), row range, Info base
enum { GROUP_STRIDE = 4, G_CUT = 0, G_R0 = 1, G_R1 = 2, G_INFO = 3 };
// forces (forces.py): Thrusters first, then Twisters (application order)
enum { FORCE_STRIDE = 8, F_TYPE = 0, F_BODY = 1, F_IDX = 2, F_STR = 5, F_MASS = 6 };
enum {
  ROW_STRIDE = 48,
  R_GROUP = 0, R_A = 1, R_B = 2, R_FN = 3, R_ONEWAY = 4, R_APOS = 5, R_AEND = 8, R_ARAD = 11,
  R_BPOS = 12, R_BEND = 15, R_BRAD = 18, R_FRIC = 19, R_ELAS = 20, R_SCALE = 21, R_THR = 22,
  R_ERP = 23,
  // extended contact functions (bx_desc row_ext): 16 floats, then the height
  // map's word offset (from o_hm) and mesh size
  R_X = 24, R_HM_OFF = 40, R_HM_M = 41,
  // a NearNeighbors cell outside the allowed mask (top_k's -inf tail)
  R_NNMASK = 42,
  // the row's NearNeighbors cell i * U + j (colliders.py:84-85), -1 for Pairs rows
  R_FLAT = 43,
};
enum {
  FK_STRIDE = 24,
  FK_BP = 0, FK_BC = 1, FK_IDX = 2, FK_ROT = 5, FK_REF = 9, FK_OFFP = 13, FK_OFFC = 16,
};
// per-env LDS record strides (floats)
// LDS record strides (words). Every stride is 4 x an odd number of words, so
// consecutive lanes' 16-byte records cover distinct bank slots: conflict-free
// for ds_read_b128 (16-lane groups, 64 banks) and ds_write_b128 (8-lane
// groups, 32 banks) when lane i touches record i (MI355X_MICROARCH.md §LDS).
// Slot regions hold parent/a-side records first, then child/b-side records,
// then one zero record: slot(j) = j, slot'(j) = n + j, zero = 2n.
enum {
  QP_STRIDE = 20,
  PREV_STRIDE = 12,
  RB_STRIDE = 12,
  ACC_STRIDE = 12,
  SLOT_STRIDE = 12,   // joint and contact slots: dp pos 3, dq rot 4, count 1
  ASLOT_STRIDE = 4,   // actuator slots: dang 3
  ROWD_STRIDE = 12    // contact row data: cpos 3, normal 3, pen, dlambda
};
enum { ACC_ICV = 0, ACC_ICA = 3, ACC_IAA = 6, ACC_DPA = 9 };

struct BlobHdr {
  int32_t N, J, K, R, G, A, substeps, D;
  int32_t num_joint_dof, n_fk, n_root_groups, L;
  float h, vexp, aexp, dt;
  float gx, gy, gz, pad0;
  // word offsets into the blob
  int32_t o_body, o_joint, o_act, o_row;
  int32_t o_jl_off, o_jl, o_al_off, o_al, o_cl_off, o_cl;
  int32_t o_base, o_fk, o_zoff, o_zpt, o_zero, o_rgroup;
  int32_t total_words;
  // per-env LDS layout (float offsets) and size
  int32_t l_qp, l_prev, l_rb, l_jslot, l_aslot, l_rowd, l_cslot, l_acc, l_ang, l_red;
  int32_t env_words;
  int32_t single;  // every lane owns <= 1 item per kind, lists <= MAXG
  int32_t act_same; // actuator a drives joint a for every a
  int32_t const_words;  // words [0, const_words) = everything the step kernels read
  int32_t NF, o_force;  // forces
  int32_t o_group, n_nn, info_rows;  // collider groups, culled groups, Info rows
  int32_t l_ract;                    // LDS: per-row NearNeighbors rank (-1 = culled)
  int32_t l_alist;                   // LDS: active rows in Info order (info_rows)
  int32_t spring;                    // dynamics_mode == legacy_spring
  int32_t o_hm;                      // height map grids
  int32_t o_hull;                    // box hulls: 8 corners, 6x4 quad points, 6 normals
  int32_t o_dangle;                  // reset: System.default_angle (num_joint_dof)
  // MULTI mode (large pbd scenes): gather tasks and the mode's LDS tail
  int32_t multi;                     // the system fits the MULTI-mode kernel
  int32_t T, o_task, o_btask;        // tasks: TASK_W slot indices each; per body BTASK_W task refs
  int32_t l_mslot, l_tslot;          // LDS: 6-word contact slots (R + two-way + 1), task partials (T+1)
  int32_t env_words_m;               // per-env LDS words in MULTI mode
  int32_t l_xact;                    // LDS: the action an env program hands System.step
  int32_t xact_words;
  int32_t o_lane;                    // SINGLE mode: the lane image (below); 0 = none
  int32_t l_arow, act_read;          // LDS: the env's action row, the words any step reads
  int32_t l_nnl, nnl_words;          // LDS: NearNeighbors per-wave pick lists (envs over several waves)
  int32_t o_bimg;                    // MULTI mode: the rows' broad-phase bounds (BI_*), 0 = none
  int32_t l_near;                    // LDS (MULTI, all-pairs scenes): the pass's near rows (R, 16-bit)
  int32_t l_jlim;                    // LDS (SINGLE, spherical kernels): each lane's joint limit rows
  int32_t m_zero;                    // MULTI: the zero contact slot (R + two-way rows)
  int32_t l_nearc;                   // LDS (MULTI): the broad phase's per-wave counts (16)
  int32_t n_cen, o_cen;              // MULTI broad phase: the capsule centres (body, offset)
  int32_t l_bimg, l_cen;             // LDS (MULTI broad phase): the rows' bounds, the centres
  int32_t o_mjh;                     // MULTI joint halves: the image (MJ_*) of lane l's joint side, 0 = none
  int32_t n_mat;                     // MULTI row tables: materials (after the collidables, o_cen / l_cen)
  int32_t l_sidx;                    // LDS (MULTI): per row its compact contact index this pass (u16, R + 1)
  int32_t l_cbuf;                    // LDS (MULTI): the penetrating rows' contacts (MCBUF x MCB_W), then their rows (u16)
  int32_t l_cnt;                     // LDS (MULTI): per-wave ballot counts (broad phase 32, listing 2 x 8)
  int32_t multi_L;                   // MULTI: threads per env (128: four envs per CU; 256)
};

// SINGLE-mode lane image: for each of 64 lanes, every constant the
// register-hoisted kernels keep (the lane's body, joint, actuator and contact
// row records, with the masses / inertias they reference, and its three
// padded gather lists), so that a lane fetches them with independent 16-byte
// loads instead of chains of dependent L2 reads (record index -> record ->
// referenced body). Word w of lane l sits at o_lane + (w / 4) * 256 + 4 * l +
// w % 4: the 16 lanes of an env read 256 contiguous bytes per load.
enum {
  LANE_IMG_LANES = 64,
  LI_BODY = 0,      // mass, inv inertia 3, pos mask 3, rot mask 3, quat mask 4
  LI_JOINT = 16,    // the lane's joint (LJ_*): lane j -> joint j
  LI_ACT = 64,      // the lane's actuator (LA_*)
  LI_ROW = 72,      // the lane's contact row (LR_*)
  LI_JL = 104,      // joint, actuator and contact gather lists, 8 entries each
  LI_AL = 112,
  LI_CL = 120,
  LI_JOINT_H = 128, // joint halves: lane l -> joint / actuator l & 7
  LI_ACT_H = 176,
  LI_JLIM = 184,    // the lane's joint's first limit row (LL_*), both mappings
  LI_JLIM_H = 192,
  LI_SIDE_H = 200,  // joint halves: this lane's side of its joint (LS_*)
  LI_JLIM12 = 216,  // the lane's joint's limit rows 1 and 2 (LL_*, 8 words each; lane j -> joint j)
  LI_ROW2 = 232,    // F_R2: the lane's second contact row (LR_*)
  LI_RIDX = 264,    // F_R2: the indices of the lane's two rows (-1: none)
  LI_CL2 = 268,     // F_C16: contact gather-list entries 8..15
  // JB (joint halves own body copies, the Ant / HalfCheetah env kernels): the
  // body record and gather lists of the lane's SIDE body (LS_BODY)
  LI_BODY_J = 276,
  LI_JL_J = 292,
  LI_AL_J = 300,
  LI_CL_J = 308,
  LANE_W = 316
};
// MULTI-mode joint halves: lane l works side (l & 8: child) of joint
// (l >> 4) * 8 + (l & 7) and that joint's actuator, the Ant kernel's halves
// in every 16-lane row of the env's 256; word w of lane l at o_mjh +
// (w / 4) * 4 * 256 + 4 * l + w % 4: the joint (LJ_*), the actuator (LA_*),
// the first limit row (LL_*), the side (LS_*)
enum { MJ_JOINT = 0, MJ_ACT = 48, MJ_JLIM = 56, MJ_SIDE = 64, MJ_W = 80, MJ_LANES = 256 };
// a joint-halves lane's side (lanes 8-15 of 16: the child's): its anchor offset,
// hinge axis and reference axis in its body's frame, that body's inverse
// inertia and mass, the side's sign (+1 parent, -1 child) and the body;
// LS_OWN: 1 on the lowest lane whose side is that body (JB: the copy that
// counts in per-body sums)
enum { LS_OFF = 0, LS_AX0 = 3, LS_AX2 = 6, LS_I = 9, LS_M = 12, LS_SG = 13, LS_BODY = 14, LS_OWN = 15 };
// a limit row [lo, hi] as the SINGLE-mode kernels test it: the
// pseudo-angles of the limits (a monotone stand-in for atan2 over (-pi, pi],
// +-3 past +-pi) and their cosines / sines
enum { LL_PLO = 0, LL_PHI = 1, LL_CLO = 2, LL_SLO = 3, LL_CHI = 4, LL_SHI = 5 };
enum {
  LJ_TYPE = 0, LJ_BP = 1, LJ_BC = 2, LJ_FREE = 3, LJ_AOFF = 4, LJ_NANG = 5, LJ_DAMP = 6,
  LJ_SP = 7, LJ_SA = 8, LJ_OFFP = 9, LJ_OFFC = 12, LJ_AXP = 15, LJ_AXC = 24, LJ_LIM = 33,
  LJ_MP = 39, LJ_MC = 40, LJ_IP = 41, LJ_IC = 44, LJ_DOF = 47  // 48 words
};
enum { LA_TYPE = 0, LA_JOINT = 1, LA_IDX = 2, LA_STR = 5 };
enum {
  LR_GROUP = 0, LR_A = 1, LR_B = 2, LR_FN = 3, LR_OW = 4, LR_APOS = 5, LR_AEND = 8,
  LR_ARAD = 11, LR_BPOS = 12, LR_BEND = 15, LR_BRAD = 18, LR_FRIC = 19, LR_ELAS = 20,
  LR_SCALE = 21, LR_THR = 22, LR_ERP = 23, LR_MA = 24, LR_MB = 25, LR_IA = 26, LR_IB = 29  // 32
};
// MULTI-mode gather tasks: a task sums <= TASK_W contact slots of one body and
// collider group; a body adds <= BTASK_W task partials (ref = task | group << 24).
// MULTI contact slots are 6 words: the linear part (position or velocity
// change, 3) and the angular part (3: the position pass's angular impulse
// before the body's one quaternion product, the velocity pass's angular
// velocity change); the count is the linear part's any-nonzero, formed where
// the task sums (slots: the compact layout below; m_zero = 2 MCAP). Task
// partials: 8 words (the two sums, the count).
enum { TASK_W = 8, BTASK_W = 8, MSLOT_STRIDE = 6, TSLOT_STRIDE = 8 };
// MULTI compact contacts (round 6). Only a penetrating row (pen > 0, or NaN)
// has a nonzero impulse (`c < 0` / `penetration > 0` masks,
// colliders.py:306-377, 584-658), so only those get contact slots: each
// pass lists them in (m, wave, lane) order (compact index y), keeps their
// contacts (cpos 3, normal 3, penetration, dlambda) in LDS (y < MCBUF) or in
// the env's slice of a global overflow buffer (MOVF_W words each), and
// writes y into the row's index word (l_sidx; 0xFFFF: no slot). The impulse
// passes run in chunks of MCAP rows: row y's a side in slot y - chunk, its b
// side in slot MCAP + y - chunk, the zero slot at 2 MCAP. A task entry is a
// row and side (row | side << 15; padding: row R, whose index stays 0xFFFF),
// resolved through l_sidx; its partial accumulates over the chunks.
enum { MCAP = 128, MCBUF = 128, MCB_W = 8, MOVF_W = 12 };
// MULTI-mode broad phase: per row two words at o_bimg + 2 r (staged in LDS
// at l_bimg once per launch): BI_W0 = centre a | centre b << 8 | flags << 16
// (<= 256 collidables), BI_W1 = (reach + 1e-4)^2 as a half float rounded up
// | Info index << 16. A capsule-capsule row whose capsule centres lie farther
// apart than reach (half segments + radii, rounded up) cannot penetrate, and
// its position / velocity updates are exact zeros. The centres are the
// distinct (body, offset) pairs of the rows' capsules, 16 bytes each at
// o_cen + 4 k: (body, offset xyz), staged at l_cen; each broad-phase pass
// places them in the world once (l_cen + 4 n_cen + 4 k) for every row that
// names them.
// The flags: bit 0 may_skip (capsule-capsule), bit 1 the row's group is
// culled (NearNeighbors), bit 2 a masked cell (R_NNMASK), bit 3 one-way,
// bits 4-7 the contact function, 8-15 the material. The Info index: a row
// of an unculled group's.
// The row tables at o_cen (uint4 units, staged at l_cen once per launch):
// 2 n_cen collidable groups ((body, offset), (end, radius)), n_mat materials
// (friction, elasticity, scale, velocity threshold), N bodies (mass, inverse
// inertia); in LDS then n_cen placed centres. Every MULTI contact pass
// assembles its rows' records from them (row_from_lds), the broad phase and
// the NearNeighbors keys take the placed centres (culled scenes, which have
// no broad phase, stage the same tables).
enum { BI_W0 = 0, BI_W1 = 1, BI_WORDS = 2 };
enum { BIF_SKIP = 1, BIF_CULL = 2, BIF_MASK = 4, BIF_OW = 8, BIF_FN_SHIFT = 4, BIF_MAT_SHIFT = 8 };
enum { HULL_STRIDE = 114, HULL_V = 0, HULL_F = 24, HULL_N = 96 };

}  // namespace bx
