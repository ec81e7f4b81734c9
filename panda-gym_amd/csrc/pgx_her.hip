/*
 * pgx_her.hip -- device HER replay ring ("future" goal relabelling) for gfx950.
 *
 * Restates stable-baselines3's HerReplayBuffer as used by the reference's
 * training (setup_training.py:176-179, replay_buffer_class=HerReplayBuffer /
 * the fork's VecHerReplayBuffer; n_sampled_goal 4 -> her_ratio 0.8):
 *   add():    SB3 HerReplayBuffer.add -- invalidate the old episode being
 *             overwritten at `pos`, ep_start[pos] = current episode start,
 *             store, and on done write the episode length over the episode.
 *   sample(): valid = flatnonzero(ep_length > 0) (slot-major, env-minor),
 *             uniform draw over valid, the first int(her_ratio*B) samples are
 *             virtual: goal = next_achieved_goal[t'] with t' uniform in
 *             [t, episode end) ("future", inclusive), reward =
 *             compute_reward(next_achieved_goal[t], goal) in float32
 *             (reach.py:84-89 on float32 arrays: utils.distance rounds in f32);
 *             dones = done * (1 - timeout).
 * Draws: Philox4x32-10, key = buffer seed, counter = (sample lo, sample hi,
 * draw lo, TAG_HER ^ draw hi); u0 = top 53 bits of words 0-1 picks the
 * transition (floor(u0 * n_valid)), u1 of words 2-3 picks t' (floor(u1 * (len - t))).
 *
 * Layout: every per-transition array is [capacity][n_envs][dim] so a slot is
 * one contiguous block (add() writes are coalesced; sample() gathers rows).
 * sample() is an HBM-bound gather: one 16-lane group per sample copies the
 * rows with consecutive lanes on consecutive floats.
 */
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/pgx.h"
#include "pgx_common.h"

namespace {

struct RingPtrs {
    float *obs, *ag, *dg, *action, *reward, *next_obs, *next_ag, *next_dg;
    uint8_t *done, *timeout;
    int32_t *ep_start, *ep_length, *cur_ep_start;
    int32_t *valid, *block_count, *n_valid;
};

struct RingDims {
    int32_t n, cap, od, ad;
};

constexpr uint32_t TAG_HER = 0x48455230u;

/* ------------------------------------------------------------------ add */
__global__ __launch_bounds__(256) void add_kernel(RingPtrs p, RingDims d, int32_t pos, pgx_transition t) {
    const int e = blockIdx.x * blockDim.x + threadIdx.x;
    const int N = d.n, C = d.cap;
    if (e >= N) return;
    const size_t se = (size_t)pos * N + e;
    /* an old episode is being overwritten: its remaining transitions become invalid */
    const int32_t old_len = p.ep_length[se];
    if (old_len > 0) {
        const int32_t end = p.ep_start[se] + old_len;
        for (int32_t k = pos; k < end; k++) p.ep_length[(size_t)(k % C) * N + e] = 0;
    }
    p.ep_start[se] = p.cur_ep_start[e];
    for (int k = 0; k < d.od; k++) {
        p.obs[se * d.od + k] = t.obs[(size_t)e * d.od + k];
        p.next_obs[se * d.od + k] = t.next_obs[(size_t)e * d.od + k];
    }
    for (int k = 0; k < 3; k++) {
        p.ag[se * 3 + k] = t.achieved_goal[(size_t)e * 3 + k];
        p.dg[se * 3 + k] = t.desired_goal[(size_t)e * 3 + k];
        p.next_ag[se * 3 + k] = t.next_achieved_goal[(size_t)e * 3 + k];
        p.next_dg[se * 3 + k] = t.next_desired_goal[(size_t)e * 3 + k];
    }
    for (int k = 0; k < d.ad; k++) p.action[se * d.ad + k] = t.action[(size_t)e * d.ad + k];
    p.reward[se] = t.reward[e];
    const uint8_t dn = t.done[e];
    p.done[se] = dn;
    p.timeout[se] = t.timeout ? t.timeout[e] : 0;
    /* the ring was written before ep_length is set below: SB3 stores then computes lengths */
    if (dn) {
        const int32_t start = p.cur_ep_start[e];
        int32_t end = (pos + 1) % C;
        if (end < start) end += C;
        const int32_t len = end - start;
        for (int32_t k = start; k < end; k++) p.ep_length[(size_t)(k % C) * N + e] = len;
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

constexpr int GROUP = 16;  /* lanes per sample */

__global__ __launch_bounds__(256) void sample_kernel(RingPtrs p, RingDims d, int64_t B, int64_t nb_virtual,
                                                     uint64_t seed, uint64_t draw, int32_t reward_type,
                                                     int32_t strategy, float thr, pgx_replay_batch o) {
    const int lane = threadIdx.x % GROUP;
    const int64_t b = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) / GROUP;
    if (b >= B) return;
    const int N = d.n, C = d.cap;
    const int32_t nv = *p.n_valid;
    if (nv <= 0) {  /* no finished episode yet: SB3 raises; mark the rows invalid */
        for (int k = lane; k < d.od; k += GROUP) o.obs[b * d.od + k] = o.next_obs[b * d.od + k] = 0.0f;
        for (int k = lane; k < d.ad; k += GROUP) o.action[b * d.ad + k] = 0.0f;
        if (lane < 3)
            o.achieved_goal[b * 3 + lane] = o.next_achieved_goal[b * 3 + lane] = o.desired_goal[b * 3 + lane] =
                o.next_desired_goal[b * 3 + lane] = 0.0f;
        if (lane == 0) {
            o.reward[b] = o.done[b] = 0.0f;
            if (o.slot) o.slot[b] = -1;
            if (o.env) o.env[b] = -1;
            if (o.goal_slot) o.goal_slot[b] = -1;
        }
        return;
    }
    uint32_t r[4];
    philox((uint32_t)b, (uint32_t)(b >> 32), (uint32_t)draw, TAG_HER ^ (uint32_t)(draw >> 32), (uint32_t)seed,
           (uint32_t)(seed >> 32), r);
    const double u0 = u53(r[0], r[1]), u1 = u53(r[2], r[3]);
    int64_t j = (int64_t)(u0 * (double)nv);
    if (j >= nv) j = nv - 1;
    const int32_t flat = p.valid[j];
    const int32_t slot = flat / N, env = flat % N;
    const size_t se = (size_t)slot * N + env;
    const bool her = b < nb_virtual;
    size_t ge = se;  /* row of the goal */
    int32_t goal_slot = -1;
    if (her) {
        const int32_t start = p.ep_start[se], len = p.ep_length[se];
        const int32_t cur = ((slot - start) % C + C) % C;
        int32_t t_in;
        if (strategy == PGX_HER_FINAL) t_in = len - 1;
        else if (strategy == PGX_HER_EPISODE) t_in = (int32_t)(u1 * (double)len);
        else t_in = cur + (int32_t)(u1 * (double)(len - cur));
        goal_slot = (t_in + start) % C;
        ge = (size_t)goal_slot * N + env;
    }
    const float* goal = her ? p.next_ag + ge * 3 : p.dg + se * 3;
    const float* ngoal = her ? p.next_ag + ge * 3 : p.next_dg + se * 3;
    /* SB3 concatenates (real, virtual): draw b < nb_virtual lands after the B - nb_virtual real rows */
    const int64_t row = her ? B - nb_virtual + b : b - nb_virtual;
    /* rows: consecutive lanes copy consecutive floats */
    for (int k = lane; k < d.od; k += GROUP) {
        o.obs[row * d.od + k] = p.obs[se * d.od + k];
        o.next_obs[row * d.od + k] = p.next_obs[se * d.od + k];
    }
    for (int k = lane; k < d.ad; k += GROUP) o.action[row * d.ad + k] = p.action[se * d.ad + k];
    if (lane < 3) {
        o.achieved_goal[row * 3 + lane] = p.ag[se * 3 + lane];
        o.next_achieved_goal[row * 3 + lane] = p.next_ag[se * 3 + lane];
        o.desired_goal[row * 3 + lane] = goal[lane];
        o.next_desired_goal[row * 3 + lane] = ngoal[lane];
    }
    if (lane == 0) {
        float rew;
        if (her) {
            rew = reward_f32(distance_f32_f32(p.next_ag + se * 3, goal), reward_type, thr);
        } else {
            rew = p.reward[se];
        }
        o.reward[row] = rew;
        o.done[row] = (float)p.done[se] * (1.0f - (float)p.timeout[se]);
        if (o.slot) o.slot[row] = slot;
        if (o.env) o.env[row] = env;
        if (o.goal_slot) o.goal_slot[row] = goal_slot;
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

int pgx_replay_create(const pgx_replay_config* cfg, int device, pgx_replay_handle* out) {
    if (!cfg || !out || cfg->n_envs <= 0 || cfg->capacity <= 1 || cfg->obs_dim <= 0 || cfg->action_dim <= 0)
        return pgx_set_error(PGX_E_INVALID, "pgx_replay_create: bad config (n_envs, capacity > 1, dims > 0)");
    if (!(cfg->her_ratio >= 0.0 && cfg->her_ratio <= 1.0))
        return pgx_set_error(PGX_E_INVALID, "pgx_replay_create: her_ratio must be in [0, 1]");
    if ((int64_t)cfg->capacity * cfg->n_envs >= (1ll << 31))
        return pgx_set_error(PGX_E_INVALID, "pgx_replay_create: capacity * n_envs must be < 2^31");
    if (cfg->reward_type != PGX_REWARD_SPARSE && cfg->reward_type != PGX_REWARD_DENSE)
        return pgx_set_error(PGX_E_INVALID, "pgx_replay_create: unknown reward_type");
    if (cfg->strategy < PGX_HER_FUTURE || cfg->strategy > PGX_HER_EPISODE)
        return pgx_set_error(PGX_E_INVALID, "pgx_replay_create: unknown goal selection strategy");
    *out = nullptr;
    if (hipSetDevice(device) != hipSuccess) return PGX_E_HIP;
    pgx_replay* h = new pgx_replay();
    h->device = device;
    h->cfg = *cfg;
    const size_t N = cfg->n_envs, C = cfg->capacity, od = cfg->obs_dim, ad = cfg->action_dim, T = N * C;
    const size_t nblocks = (T + SCAN_BLOCK - 1) / SCAN_BLOCK;
    auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
    size_t sizes[] = {T * od * 4, T * 12, T * 12, T * ad * 4, T * 4, T * od * 4, T * 12, T * 12, T, T,
                      T * 4, T * 4, N * 4, T * 4, nblocks * 4, 4};
    size_t off[16], total = 0;
    for (int i = 0; i < 16; i++) { off[i] = total; total = al(total + sizes[i]); }
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
    p.obs = (float*)(b + off[0]); p.ag = (float*)(b + off[1]); p.dg = (float*)(b + off[2]);
    p.action = (float*)(b + off[3]); p.reward = (float*)(b + off[4]); p.next_obs = (float*)(b + off[5]);
    p.next_ag = (float*)(b + off[6]); p.next_dg = (float*)(b + off[7]); p.done = (uint8_t*)(b + off[8]);
    p.timeout = (uint8_t*)(b + off[9]); p.ep_start = (int32_t*)(b + off[10]); p.ep_length = (int32_t*)(b + off[11]);
    p.cur_ep_start = (int32_t*)(b + off[12]); p.valid = (int32_t*)(b + off[13]);
    p.block_count = (int32_t*)(b + off[14]); p.n_valid = (int32_t*)(b + off[15]);
    h->d = RingDims{cfg->n_envs, cfg->capacity, cfg->obs_dim, cfg->action_dim};
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
    const int N = h->d.n;
    hipLaunchKernelGGL(add_kernel, dim3((N + 255) / 256), dim3(256), 0, (hipStream_t)stream, h->p, h->d, h->pos, *t);
    if (hipGetLastError() != hipSuccess) return pgx_set_error(PGX_E_HIP, "pgx_replay_add: launch failed");
    h->pos = (h->pos + 1) % h->d.cap;
    h->added += 1;
    return PGX_OK;
}

int64_t pgx_replay_size(pgx_replay_handle h) { return h ? h->added : PGX_E_INVALID; }

int pgx_replay_sample(pgx_replay_handle h, int64_t batch, uint64_t draw, pgx_replay_batch* out, void* stream) {
    if (!h || !out || batch <= 0 || batch > (1ll << 26))
        return pgx_set_error(PGX_E_INVALID, "pgx_replay_sample: null handle or batch not in [1, 2^26]");
    if (!out->obs || !out->achieved_goal || !out->desired_goal || !out->action || !out->reward || !out->next_obs ||
        !out->next_achieved_goal || !out->next_desired_goal || !out->done)
        return pgx_set_error(PGX_E_INVALID, "pgx_replay_sample: null output pointer");
    if (h->added == 0) return pgx_set_error(PGX_E_INVALID, "pgx_replay_sample: buffer is empty");
    hipStream_t st = (hipStream_t)stream;
    const int64_t total = (int64_t)h->d.n * h->d.cap;
    const int32_t nblocks = (int32_t)((total + SCAN_BLOCK - 1) / SCAN_BLOCK);
    hipLaunchKernelGGL(count_kernel, dim3(nblocks), dim3(SCAN_BLOCK), 0, st, h->p, total);
    hipLaunchKernelGGL(scan_blocks_kernel, dim3(1), dim3(1024), 0, st, h->p, nblocks);
    hipLaunchKernelGGL(scatter_kernel, dim3(nblocks), dim3(SCAN_BLOCK), 0, st, h->p, total);
    const int64_t nb_virtual = (int64_t)(h->cfg.her_ratio * (double)batch);
    const int64_t threads = batch * GROUP;
    hipLaunchKernelGGL(sample_kernel, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0, st, h->p, h->d, batch,
                       nb_virtual, h->cfg.seed, draw, h->cfg.reward_type, h->cfg.strategy, (float)h->cfg.distance_threshold, *out);
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
