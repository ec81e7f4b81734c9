/*
 * pgx_her.hip -- device HER replay ring (goal relabelling) for gfx950.
 *
 * Restates stable-baselines3's HerReplayBuffer as used by the reference's
 * training (setup_training.py:14,176-179, classes/train_config.py:15;
 * n_sampled_goal 4 -> her_ratio 0.8):
 *   add():    SB3 HerReplayBuffer.add -- invalidate the old episode being
 *             overwritten at `pos`, ep_start[pos] = current episode start,
 *             store, and on done write the episode length over the episode;
 *             then refresh valid = flatnonzero(ep_length > 0) (slot-major,
 *             env-minor), the only state sample() depends on besides the ring.
 *   sample(): uniform draw over valid; the first int(her_ratio*B) draws are
 *             virtual: goal = next_achieved_goal[t'] with t' from the episode
 *             of t ("future": uniform in [t, end)), reward =
 *             compute_reward(next_achieved_goal[t], goal) in float32
 *             (reach.py:84-89 on float32 arrays); dones = done * (1 - timeout);
 *             output rows real first, then virtual (SB3 concatenation order).
 * Draws: Philox4x32-10, key = buffer seed, counter = (sample lo, sample hi,
 * draw lo, TAG_HER ^ draw hi); u0 = top 53 bits of words 0-1 picks the
 * transition (floor(u0 * n_valid)), u1 of words 2-3 picks t'.
 *
 * Layout (HBM): one record of R floats per (slot, env), R = round_up(row_dim
 * + 2, 32) -- the batch row (pgx.h) followed by the transition's ep_start and
 * ep_length -- so a sampled transition is R*4 contiguous bytes (2 x 128 B
 * lines for PickAndPlace) instead of a dozen scattered field rows.  Dense
 * ep_start/ep_length [C][N] arrays carry SB3's bookkeeping (compaction reads
 * 4 B per transition); the record copy of ep_length is refreshed whenever an
 * episode completes and only read for transitions the dense array marks valid.
 *
 * sample(): one wave per 64 draws.  Phase 1: lane i draws sample i (Philox,
 * valid-list lookup, episode fields, goal, relabelled reward) into LDS.
 * Phase 2: 16-lane groups copy 4 records at a time with float4 loads/stores,
 * patching desired goals and reward of the relabelled rows.
 */
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <cstdlib>

#include "../../include/pgx.h"
#include "pgx_common.h"

namespace {

constexpr uint32_t TAG_HER = 0x48455230u;
constexpr int GROUP = 16;  /* lanes per record copy (float4 each) */

struct RingPtrs {
    float* rec;                 /* [C][N][R] */
    int32_t *ep_start, *ep_length, *cur_ep_start;
    int32_t *valid, *block_count, *n_valid;
};

/* field offsets inside a row / record (floats) */
struct RingDims {
    int32_t n, cap, od, ad;
    int32_t R, S;               /* record stride, batch row stride */
    int32_t ag, dg, act, rew, nobs, nag, ndg, done, eps, epl;
};

RingDims make_dims(const pgx_replay_config& c) {
    RingDims d{};
    d.n = c.n_envs;
    d.cap = c.capacity;
    d.od = c.obs_dim;
    d.ad = c.action_dim;
    d.ag = d.od;
    d.dg = d.ag + 3;
    d.act = d.dg + 3;
    d.rew = d.act + d.ad;
    d.nobs = d.rew + 1;
    d.nag = d.nobs + d.od;
    d.ndg = d.nag + 3;
    d.done = d.ndg + 3;
    d.eps = d.done + 1;        /* == row_dim */
    d.epl = d.eps + 1;
    d.S = (d.eps + 3) & ~3;
    d.R = (d.epl + 1 + 31) & ~31;
    return d;
}

__device__ __forceinline__ float ibits(int32_t v) { return __int_as_float(v); }
__device__ __forceinline__ int32_t fbits(float v) { return __float_as_int(v); }

/* ------------------------------------------------------------------ add */
/* value of record float f for env e of transition t */
__device__ __forceinline__ float record_value(const RingDims& d, const pgx_transition& t, int e, int f, float dones,
                                              int32_t cur, int32_t len) {
    if (f < d.ag) return t.obs[(size_t)e * d.od + f];
    if (f < d.dg) return t.achieved_goal[(size_t)e * 3 + (f - d.ag)];
    if (f < d.act) return t.desired_goal[(size_t)e * 3 + (f - d.dg)];
    if (f < d.rew) return t.action[(size_t)e * d.ad + (f - d.act)];
    if (f == d.rew) return t.reward[e];
    if (f < d.nag) return t.next_obs[(size_t)e * d.od + (f - d.nobs)];
    if (f < d.ndg) return t.next_achieved_goal[(size_t)e * 3 + (f - d.nag)];
    if (f < d.done) return t.next_desired_goal[(size_t)e * 3 + (f - d.ndg)];
    if (f == d.done) return dones;
    if (f == d.eps) return ibits(cur);
    if (f == d.epl) return ibits(len);
    return 0.0f;
}

__global__ __launch_bounds__(64) void add_kernel(RingPtrs p, RingDims d, int32_t pos, pgx_transition t) {
    const int g = threadIdx.x % GROUP;
    const int e = blockIdx.x * (64 / GROUP) + threadIdx.x / GROUP;
    const int N = d.n, C = d.cap;
    if (e >= N) return;
    const size_t se = (size_t)pos * N + e;
    const int32_t cur = p.cur_ep_start[e];
    const bool dn = t.done[e] != 0;
    const bool to = t.timeout ? t.timeout[e] != 0 : false;
    int32_t end = (pos + 1) % C;
    if (end < cur) end += C;
    const int32_t len = dn ? end - cur : 0;
    /* SB3 stores done and timeout; sample() only ever uses done * (1 - timeout) */
    const float dones = (float)dn * (1.0f - (float)to);
    float* rec = p.rec + se * d.R;
    for (int c = g; 4 * c < d.R; c += GROUP) {
        float4 v;
        v.x = record_value(d, t, e, 4 * c + 0, dones, cur, len);
        v.y = record_value(d, t, e, 4 * c + 1, dones, cur, len);
        v.z = record_value(d, t, e, 4 * c + 2, dones, cur, len);
        v.w = record_value(d, t, e, 4 * c + 3, dones, cur, len);
        *reinterpret_cast<float4*>(rec + 4 * c) = v;
    }
    if (g != 0) return;
    /* an old episode is being overwritten: its remaining transitions become invalid */
    const int32_t old_len = p.ep_length[se];
    if (old_len > 0) {
        const int32_t old_end = p.ep_start[se] + old_len;
        for (int32_t k = pos; k < old_end; k++) p.ep_length[(size_t)(k % C) * N + e] = 0;
    }
    p.ep_start[se] = cur;
    if (dn) {  /* SB3 _compute_episode_length: the new episode spans [cur, end) */
        for (int32_t k = cur; k < end; k++) {
            const size_t sk = (size_t)(k % C) * N + e;
            p.ep_length[sk] = len;
            if (k % C != pos) p.rec[sk * d.R + d.epl] = ibits(len);  /* own record written above */
        }
        p.cur_ep_start[e] = (pos + 1) % C;
    }
}

/* ------------------------------------------- ordered compaction of ep_length > 0 */
constexpr int SCAN_BLOCK = 1024;

__global__ __launch_bounds__(SCAN_BLOCK) void count_kernel(RingPtrs p, int64_t total) {
    __shared__ int32_t s[SCAN_BLOCK / 64];
    const int64_t i = (int64_t)blockIdx.x * SCAN_BLOCK + threadIdx.x;
    const int v = (i < total && p.ep_length[i] > 0) ? 1 : 0;
    const int w = __popcll(__ballot(v));
    if ((threadIdx.x & 63) == 0) s[threadIdx.x >> 6] = w;
    __syncthreads();
    if (threadIdx.x == 0) {
        int c = 0;
        for (int k = 0; k < SCAN_BLOCK / 64; k++) c += s[k];
        p.block_count[blockIdx.x] = c;
    }
}

/* exclusive scan of the block counts in one workgroup (block_count -> offsets, n_valid) */
__global__ __launch_bounds__(1024) void scan_blocks_kernel(RingPtrs p, int32_t nblocks) {
    __shared__ int32_t s[1024];
    int32_t carry = 0;
    for (int32_t base = 0; base < nblocks; base += 1024) {
        const int32_t i = base + threadIdx.x;
        const int32_t v = i < nblocks ? p.block_count[i] : 0;
        s[threadIdx.x] = v;
        __syncthreads();
        for (int off = 1; off < 1024; off <<= 1) {
            int32_t t = threadIdx.x >= off ? s[threadIdx.x - off] : 0;
            __syncthreads();
            s[threadIdx.x] += t;
            __syncthreads();
        }
        if (i < nblocks) p.block_count[i] = carry + s[threadIdx.x] - v;
        carry += s[1023];
        __syncthreads();
    }
    if (threadIdx.x == 0) *p.n_valid = carry;
}

__global__ __launch_bounds__(SCAN_BLOCK) void scatter_kernel(RingPtrs p, int64_t total) {
    __shared__ int32_t s[SCAN_BLOCK / 64];
    const int64_t i = (int64_t)blockIdx.x * SCAN_BLOCK + threadIdx.x;
    const int v = (i < total && p.ep_length[i] > 0) ? 1 : 0;
    const uint64_t bal = __ballot(v);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    if (lane == 0) s[wave] = __popcll(bal);
    __syncthreads();
    if (threadIdx.x == 0) {
        int c = 0;
        for (int k = 0; k < SCAN_BLOCK / 64; k++) { int t = s[k]; s[k] = c; c += t; }
    }
    __syncthreads();
    if (v) {
        const int before = __popcll(bal & ((1ull << lane) - 1ull));
        p.valid[p.block_count[blockIdx.x] + s[wave] + before] = (int32_t)i;
    }
}

/* ---------------------------------------------------------------- sample */
struct Draw {
    int64_t rec;    /* record index (slot * N + env), -1: no valid transition */
    int64_t row;    /* output row */
    float goal[3];
    float reward;
    int32_t her;
    int32_t pad;
};

__global__ __launch_bounds__(64) void sample_kernel(RingPtrs p, RingDims d, int64_t B, int64_t nb_virtual,
                                                    uint64_t seed, uint64_t draw, int32_t reward_type,
                                                    int32_t strategy, float thr, pgx_replay_batch o) {
    __shared__ Draw dr[64];
    const int lane = threadIdx.x;
    const int64_t b0 = (int64_t)blockIdx.x * 64;
    const int N = d.n, C = d.cap;
    const int32_t nv = *p.n_valid;
    /* phase 1: lane `lane` draws sample b0 + lane */
    {
        const int64_t b = b0 + lane;
        Draw w{};
        w.rec = -1;
        if (b < B) {
            const bool her = b < nb_virtual;
            w.row = her ? B - nb_virtual + b : b - nb_virtual;
            w.her = her;
            int32_t slot = -1, env = -1, goal_slot = -1;
            if (nv > 0) {
                uint32_t r[4];
                philox((uint32_t)b, (uint32_t)(b >> 32), (uint32_t)draw, TAG_HER ^ (uint32_t)(draw >> 32),
                       (uint32_t)seed, (uint32_t)(seed >> 32), r);
                const double u0 = u53(r[0], r[1]), u1 = u53(r[2], r[3]);
                int64_t j = (int64_t)(u0 * (double)nv);
                if (j >= nv) j = nv - 1;
                const int32_t flat = p.valid[j];
                slot = flat / N;
                env = flat % N;
                w.rec = flat;
                if (her) {
                    const float* rc = p.rec + (size_t)flat * d.R;
                    const int32_t start = fbits(rc[d.eps]), len = fbits(rc[d.epl]);
                    const int32_t cur = ((slot - start) % C + C) % C;
                    int32_t t_in;
                    if (strategy == PGX_HER_FINAL) t_in = len - 1;
                    else if (strategy == PGX_HER_EPISODE) t_in = (int32_t)(u1 * (double)len);
                    else t_in = cur + (int32_t)(u1 * (double)(len - cur));
                    goal_slot = (t_in + start) % C;
                    const float* gr = p.rec + ((size_t)goal_slot * N + env) * d.R + d.nag;
                    w.goal[0] = gr[0]; w.goal[1] = gr[1]; w.goal[2] = gr[2];
                    w.reward = reward_f32(distance_f32_f32(rc + d.nag, w.goal), reward_type, thr);
                }
            }
            if (o.slot) o.slot[w.row] = slot;
            if (o.env) o.env[w.row] = env;
            if (o.goal_slot) o.goal_slot[w.row] = goal_slot;
        }
        dr[lane] = w;
    }
    __syncthreads();
    /* phase 2: 16-lane groups copy 4 records per step; the loads of UNROLL steps are issued
     * before their stores, so each lane keeps several 16-B reads in flight */
    const int g = lane % GROUP;
    constexpr int UNROLL = 8;
    auto fetch = [&](const Draw& w, int c) {
        float4 v = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
        if (w.rec >= 0 && 4 * c < d.S) v = *reinterpret_cast<const float4*>(p.rec + w.rec * d.R + 4 * c);
        return v;
    };
    auto finish = [&](const Draw& w, int c, float4 v) {
        if (4 * c >= d.S) return;
        float* vv = reinterpret_cast<float*>(&v);
        if (w.rec >= 0 && w.her) {
#pragma unroll
            for (int k = 0; k < 4; k++) {
                const int f = 4 * c + k;
                if (f >= d.dg && f < d.dg + 3) vv[k] = w.goal[f - d.dg];
                else if (f >= d.ndg && f < d.ndg + 3) vv[k] = w.goal[f - d.ndg];
                else if (f == d.rew) vv[k] = w.reward;
            }
        }
        /* the record's ep_start/ep_length may share the last float4: not part of a row */
#pragma unroll
        for (int k = 0; k < 4; k++)
            if (4 * c + k >= d.eps) vv[k] = 0.0f;
        /* streaming store: the batch is written once and read by the learner later */
        typedef float f4v __attribute__((ext_vector_type(4)));
        const f4v nv4 = {v.x, v.y, v.z, v.w};
        __builtin_nontemporal_store(nv4, reinterpret_cast<f4v*>(o.rows + w.row * d.S + 4 * c));
    };
    for (int c = g; 4 * c < d.S; c += GROUP) {
        for (int s0 = lane / GROUP; s0 < 64; s0 += UNROLL * (64 / GROUP)) {
            float4 v[UNROLL];
#pragma unroll
            for (int u = 0; u < UNROLL; u++) {
                const int s = s0 + u * (64 / GROUP);
                v[u] = (s < 64 && b0 + s < B) ? fetch(dr[s], c) : make_float4(0.0f, 0.0f, 0.0f, 0.0f);
            }
#pragma unroll
            for (int u = 0; u < UNROLL; u++) {
                const int s = s0 + u * (64 / GROUP);
                if (s < 64 && b0 + s < B) finish(dr[s], c, v[u]);
            }
        }
    }
}

/* sample(), records of at most 16 float4 columns (the batch row plus ep_start / ep_length: every
 * task but ReachAO's 56-float observation): each record is read from HBM once.  Phase A: lane i
 * draws sample i (Philox, valid-list lookup).  Phase B: 16-lane groups load the 64 records into
 * registers (lane c of a group holds column c of 16 records, one float4 load each) and stage the
 * fields the relabelling reads -- next_achieved_goal, ep_start, ep_length -- in LDS.  Phase C:
 * lane i relabels sample i (future goal gather, reward) from the staged fields.  Phase D: the
 * groups patch desired goals and reward and store the rows.  (sample_kernel above reads the
 * episode fields in its first phase and the record again in its copy: the record's second line
 * twice, 556 B of reads per PickAndPlace sample for 358 B of data, profiles/pmc_sample_kernel.json
 * of round 4.)  Same draws, same arithmetic: the rows are bit-identical. */
constexpr int REG_COLS = 16;
/* SPB: samples per 64-lane block (lane i < SPB draws sample i); each lane holds SPB / 4 records'
 * columns in registers */
template <int SPB>
__global__ __launch_bounds__(64) void sample_kernel_reg(RingPtrs p, RingDims d, int64_t B, int64_t nb_virtual,
                                                        uint64_t seed, uint64_t draw, int32_t reward_type,
                                                        int32_t strategy, float thr, pgx_replay_batch o) {
    __shared__ Draw dr[SPB];
    __shared__ float stg[SPB][6];   /* next_achieved_goal [3], ep_start, ep_length (bits) */
    const int lane = threadIdx.x;
    const int64_t b0 = (int64_t)blockIdx.x * SPB;
    const int N = d.n, C = d.cap;
    const int32_t nv = *p.n_valid;
    const int ncol = (d.epl + 4) / 4;   /* columns holding the row and the episode fields */
    /* phase A */
    const int64_t b = b0 + lane;
    double u1 = 0.0;
    if (lane < SPB) {
        Draw w{};
        w.rec = -1;
        if (b < B) {
            const bool her = b < nb_virtual;
            w.row = her ? B - nb_virtual + b : b - nb_virtual;
            w.her = her;
            if (nv > 0) {
                uint32_t r[4];
                philox((uint32_t)b, (uint32_t)(b >> 32), (uint32_t)draw, TAG_HER ^ (uint32_t)(draw >> 32),
                       (uint32_t)seed, (uint32_t)(seed >> 32), r);
                const double u0 = u53(r[0], r[1]);
                u1 = u53(r[2], r[3]);
                int64_t j = (int64_t)(u0 * (double)nv);
                if (j >= nv) j = nv - 1;
                w.rec = p.valid[j];
            }
        }
        dr[lane] = w;
    }
    __syncthreads();
    /* phase B: lane 16 q + c holds column c of records q, q + 4, ..., q + SPB - 4 */
    const int c = lane % GROUP, q = lane / GROUP;
    float4 v[SPB / (64 / GROUP)];
#pragma unroll
    for (int k = 0; k < SPB / (64 / GROUP); k++) {
        const int sm = q + k * (64 / GROUP);
        const int64_t rec = dr[sm].rec;
        v[k] = (c < ncol && rec >= 0 && b0 + sm < B) ? *reinterpret_cast<const float4*>(p.rec + rec * d.R + 4 * c)
                                                    : make_float4(0.0f, 0.0f, 0.0f, 0.0f);
        const float vv[4] = {v[k].x, v[k].y, v[k].z, v[k].w};
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const int f = 4 * c + u;
            if (f >= d.nag && f < d.nag + 3) stg[sm][f - d.nag] = vv[u];
            if (f == d.eps) stg[sm][3] = vv[u];
            if (f == d.epl) stg[sm][4] = vv[u];
        }
    }
    __syncthreads();
    /* phase C: lane i relabels sample i */
    if (lane < SPB && b < B) {
        Draw& w = dr[lane];
        int32_t slot = -1, env = -1, goal_slot = -1;
        if (w.rec >= 0) {
            const int32_t flat = (int32_t)w.rec;
            slot = flat / N;
            env = flat % N;
            if (w.her) {
                const int32_t start = fbits(stg[lane][3]), len = fbits(stg[lane][4]);
                const int32_t cur = ((slot - start) % C + C) % C;
                int32_t t_in;
                if (strategy == PGX_HER_FINAL) t_in = len - 1;
                else if (strategy == PGX_HER_EPISODE) t_in = (int32_t)(u1 * (double)len);
                else t_in = cur + (int32_t)(u1 * (double)(len - cur));
                goal_slot = (t_in + start) % C;
                const float* gr = p.rec + ((size_t)goal_slot * N + env) * d.R + d.nag;
                w.goal[0] = gr[0]; w.goal[1] = gr[1]; w.goal[2] = gr[2];
                const float nag[3] = {stg[lane][0], stg[lane][1], stg[lane][2]};
                w.reward = reward_f32(distance_f32_f32(nag, w.goal), reward_type, thr);
            }
        }
        if (o.slot) o.slot[w.row] = slot;
        if (o.env) o.env[w.row] = env;
        if (o.goal_slot) o.goal_slot[w.row] = goal_slot;
    }
    __syncthreads();
    /* phase D: patch and store (as sample_kernel's finish) */
    typedef float f4v __attribute__((ext_vector_type(4)));
#pragma unroll
    for (int k = 0; k < SPB / (64 / GROUP); k++) {
        const int sm = q + k * (64 / GROUP);
        if (4 * c >= d.S || b0 + sm >= B) continue;
        const Draw& w = dr[sm];
        float vv[4] = {v[k].x, v[k].y, v[k].z, v[k].w};
        if (w.rec >= 0 && w.her) {
#pragma unroll
            for (int u = 0; u < 4; u++) {
                const int f = 4 * c + u;
                if (f >= d.dg && f < d.dg + 3) vv[u] = w.goal[f - d.dg];
                else if (f >= d.ndg && f < d.ndg + 3) vv[u] = w.goal[f - d.ndg];
                else if (f == d.rew) vv[u] = w.reward;
            }
        }
#pragma unroll
        for (int u = 0; u < 4; u++)
            if (4 * c + u >= d.eps) vv[u] = 0.0f;
        const f4v nv4 = {vv[0], vv[1], vv[2], vv[3]};
        __builtin_nontemporal_store(nv4, reinterpret_cast<f4v*>(o.rows + w.row * d.S + 4 * c));
    }
}

}  // namespace

struct pgx_replay {
    int device;
    pgx_replay_config cfg;
    RingPtrs p;
    RingDims d;
    void* blob;
    int32_t pos;
    int64_t added;
};

int pgx_set_error(int code, const char* msg);  /* pgx_api.cpp: sets pgx_last_error() */

extern "C" {

int pgx_replay_row_dim(const pgx_replay_config* cfg) {
    if (!cfg || cfg->obs_dim <= 0 || cfg->action_dim <= 0) return PGX_E_INVALID;
    return make_dims(*cfg).eps;
}

int pgx_replay_row_stride(const pgx_replay_config* cfg) {
    if (!cfg || cfg->obs_dim <= 0 || cfg->action_dim <= 0) return PGX_E_INVALID;
    return make_dims(*cfg).S;
}

int pgx_replay_create(const pgx_replay_config* cfg, int device, pgx_replay_handle* out) {
    if (!cfg || !out || cfg->n_envs <= 0 || cfg->capacity <= 1 || cfg->obs_dim <= 0 || cfg->action_dim <= 0)
        return pgx_set_error(PGX_E_INVALID, "pgx_replay_create: bad config (n_envs, capacity > 1, dims > 0)");
    if (!(cfg->her_ratio >= 0.0 && cfg->her_ratio <= 1.0))
        return pgx_set_error(PGX_E_INVALID, "pgx_replay_create: her_ratio must be in [0, 1]");
    if ((int64_t)cfg->capacity * cfg->n_envs >= (1ll << 31))
        return pgx_set_error(PGX_E_INVALID, "pgx_replay_create: capacity * n_envs must be < 2^31");
    if (cfg->reward_type != PGX_REWARD_SPARSE && cfg->reward_type != PGX_REWARD_DENSE &&
        cfg->reward_type != PGX_REWARD_SPARSE_AO)
        return pgx_set_error(PGX_E_INVALID, "pgx_replay_create: unknown reward_type");
    if (cfg->strategy < PGX_HER_FUTURE || cfg->strategy > PGX_HER_EPISODE)
        return pgx_set_error(PGX_E_INVALID, "pgx_replay_create: unknown goal selection strategy");
    *out = nullptr;
    if (hipSetDevice(device) != hipSuccess) return pgx_set_error(PGX_E_HIP, "pgx_replay_create: hipSetDevice");
    pgx_replay* h = new pgx_replay();
    h->device = device;
    h->cfg = *cfg;
    h->d = make_dims(*cfg);
    const size_t N = cfg->n_envs, C = cfg->capacity, T = N * C;
    const size_t nblocks = (T + SCAN_BLOCK - 1) / SCAN_BLOCK;
    auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
    const size_t sizes[] = {T * h->d.R * 4, T * 4, T * 4, N * 4, T * 4, nblocks * 4, 4};
    size_t off[7], total = 0;
    for (int i = 0; i < 7; i++) { off[i] = total; total = al(total + sizes[i]); }
    if (hipMalloc(&h->blob, total) != hipSuccess) {
        delete h;
        return pgx_set_error(PGX_E_NOMEM, "pgx_replay_create: hipMalloc failed");
    }
    if (hipMemset(h->blob, 0, total) != hipSuccess || hipDeviceSynchronize() != hipSuccess) {
        (void)hipFree(h->blob);
        delete h;
        return pgx_set_error(PGX_E_HIP, "pgx_replay_create: hipMemset failed");
    }
    char* b = (char*)h->blob;
    RingPtrs& p = h->p;
    p.rec = (float*)(b + off[0]);
    p.ep_start = (int32_t*)(b + off[1]);
    p.ep_length = (int32_t*)(b + off[2]);
    p.cur_ep_start = (int32_t*)(b + off[3]);
    p.valid = (int32_t*)(b + off[4]);
    p.block_count = (int32_t*)(b + off[5]);
    p.n_valid = (int32_t*)(b + off[6]);
    h->pos = 0;
    h->added = 0;
    *out = h;
    return PGX_OK;
}

void pgx_replay_destroy(pgx_replay_handle h) {
    if (!h) return;
    (void)hipSetDevice(h->device);
    (void)hipFree(h->blob);
    delete h;
}

int pgx_replay_add(pgx_replay_handle h, const pgx_transition* t, void* stream) {
    if (!h || !t || !t->obs || !t->achieved_goal || !t->desired_goal || !t->action || !t->reward || !t->next_obs ||
        !t->next_achieved_goal || !t->next_desired_goal || !t->done)
        return pgx_set_error(PGX_E_INVALID, "pgx_replay_add: null handle or transition pointer");
    hipStream_t st = (hipStream_t)stream;
    const int N = h->d.n;
    const int per_block = 64 / GROUP;
    hipLaunchKernelGGL(add_kernel, dim3((N + per_block - 1) / per_block), dim3(64), 0, st, h->p, h->d, h->pos, *t);
    const int64_t total = (int64_t)h->d.n * h->d.cap;
    const int32_t nblocks = (int32_t)((total + SCAN_BLOCK - 1) / SCAN_BLOCK);
    hipLaunchKernelGGL(count_kernel, dim3(nblocks), dim3(SCAN_BLOCK), 0, st, h->p, total);
    hipLaunchKernelGGL(scan_blocks_kernel, dim3(1), dim3(1024), 0, st, h->p, nblocks);
    hipLaunchKernelGGL(scatter_kernel, dim3(nblocks), dim3(SCAN_BLOCK), 0, st, h->p, total);
    if (hipGetLastError() != hipSuccess) return pgx_set_error(PGX_E_HIP, "pgx_replay_add: launch failed");
    h->pos = (h->pos + 1) % h->d.cap;
    h->added += 1;
    return PGX_OK;
}

int64_t pgx_replay_size(pgx_replay_handle h) { return h ? h->added : PGX_E_INVALID; }

int pgx_replay_sample(pgx_replay_handle h, int64_t batch, uint64_t draw, pgx_replay_batch* out, void* stream) {
    if (!h || !out || batch <= 0 || batch > (1ll << 26))
        return pgx_set_error(PGX_E_INVALID, "pgx_replay_sample: null handle or batch not in [1, 2^26]");
    if (!out->rows) return pgx_set_error(PGX_E_INVALID, "pgx_replay_sample: null rows pointer");
    if (((uintptr_t)out->rows & 15) != 0) return pgx_set_error(PGX_E_INVALID, "pgx_replay_sample: rows not 16 B aligned");
    if (h->added == 0) return pgx_set_error(PGX_E_INVALID, "pgx_replay_sample: buffer is empty");
    const int64_t nb_virtual = (int64_t)(h->cfg.her_ratio * (double)batch);
    const char* spb = std::getenv("PGX_HER_SPB");
    if ((h->d.epl + 4) / 4 <= REG_COLS && !std::getenv("PGX_HER_TWO_PASS")) {   /* records read once */
        if (spb && std::atoi(spb) == 64)
            hipLaunchKernelGGL(sample_kernel_reg<64>, dim3((unsigned)((batch + 63) / 64)), dim3(64), 0,
                               (hipStream_t)stream, h->p, h->d, batch, nb_virtual, h->cfg.seed, draw,
                               h->cfg.reward_type, h->cfg.strategy, (float)h->cfg.distance_threshold, *out);
        else
            hipLaunchKernelGGL(sample_kernel_reg<32>, dim3((unsigned)((batch + 31) / 32)), dim3(64), 0,
                               (hipStream_t)stream, h->p, h->d, batch, nb_virtual, h->cfg.seed, draw,
                               h->cfg.reward_type, h->cfg.strategy, (float)h->cfg.distance_threshold, *out);
    }
    else   /* wider records (ReachAO's 56-float observation) */
        hipLaunchKernelGGL(sample_kernel, dim3((unsigned)((batch + 63) / 64)), dim3(64), 0, (hipStream_t)stream, h->p,
                           h->d, batch, nb_virtual, h->cfg.seed, draw, h->cfg.reward_type, h->cfg.strategy,
                           (float)h->cfg.distance_threshold, *out);
    return hipGetLastError() == hipSuccess ? PGX_OK : pgx_set_error(PGX_E_HIP, "pgx_replay_sample: launch failed");
}

int pgx_replay_episode_arrays(pgx_replay_handle h, int32_t** ep_start, int32_t** ep_length, int32_t** n_valid) {
    if (!h || !ep_start || !ep_length || !n_valid) return PGX_E_INVALID;
    *ep_start = h->p.ep_start;
    *ep_length = h->p.ep_length;
    *n_valid = h->p.n_valid;
    return PGX_OK;
}

}  // extern "C"
