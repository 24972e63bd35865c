// Synthetic device-resident vectorised environments (the reference's envs are
// gym/ALE/MuJoCo processes behind SB3 SubprocVecEnv pipes, env.py:7-12 —
// unavailable offline and the one process boundary of its hot loop).  Every
// draw is Philox4x32-10 keyed by the seed with counter (block, GLOBAL env id,
// step, action), so a rank holding envs [off, off+n) produces exactly the
// slice a single GPU would: sharding never changes the data.  oracle/philox.py
// is the numpy twin used by the parity tests.
//
// Atari: (N, 4, 84, 84) uint8 frame stacks, newest frame last; on done the
// stack is zeroed and the new frame placed last (VecFrameStack auto-reset,
// .ipynb_checkpoints/env-checkpoint.py:16-17).  reward ~ Bernoulli(p_reward),
// done ~ Bernoulli(p_done).  Traffic per env-step: 3 frames read + 4 written.
#include "common.h"
#include "philox.h"

namespace {

constexpr int FRAME = 84 * 84;
constexpr int CHUNKS = FRAME / 16;  // 441
constexpr uint32_t EVENT_BLOCK = 0xFFFFFFFFu;
constexpr uint32_t RESET_ACTION = 0xFFFFFFFFu;

struct Episode {
    float* ep_ret;
    int32_t* ep_len;
    float* done_ret;  // nullable: return of the episode that ended at this step, NaN otherwise
    int32_t* done_len;
};

__device__ inline void episode_update(const Episode& ep, long long n, float rew, bool done) {
    if (!ep.ep_ret) return;
    const float r = ep.ep_ret[n] + rew;
    const int l = ep.ep_len[n] + 1;
    if (ep.done_ret) ep.done_ret[n] = done ? r : __builtin_nanf("");
    if (ep.done_len) ep.done_len[n] = done ? l : 0;
    ep.ep_ret[n] = done ? 0.f : r;
    ep.ep_len[n] = done ? 0 : l;
}

__global__ void __launch_bounds__(256) atari_reset_kernel(uint8_t* __restrict__ obs, long long env_offset, uint32_t k0,
                                                          uint32_t k1, Episode ep) {
    const long long n = blockIdx.x;
    const uint32_t gid = (uint32_t)(env_offset + n);
    uint4* o = reinterpret_cast<uint4*>(obs + n * 4LL * FRAME);
    for (int c = threadIdx.x; c < CHUNKS; c += blockDim.x) {
        const ppox::u32x4 w = ppox::philox4x32_10(ppox::u32x4{(uint32_t)c, gid, 0u, RESET_ACTION}, k0, k1);
        const uint4 z = make_uint4(0, 0, 0, 0);
        o[c] = z;
        o[CHUNKS + c] = z;
        o[2 * CHUNKS + c] = z;
        o[3 * CHUNKS + c] = make_uint4(w.x, w.y, w.z, w.w);
    }
    if (threadIdx.x == 0 && ep.ep_ret) {
        ep.ep_ret[n] = 0.f;
        ep.ep_len[n] = 0;
    }
}

__global__ void __launch_bounds__(256) atari_step_kernel(const uint8_t* __restrict__ in, uint8_t* __restrict__ out,
                                                         const int32_t* __restrict__ actions, long long env_offset,
                                                         uint32_t k0, uint32_t k1, uint32_t step,
                                                         const long long* __restrict__ sbase, float p_reward,
                                                         float p_done, float* __restrict__ rewards,
                                                         uint8_t* __restrict__ dones, Episode ep) {
    const long long n = blockIdx.x;
    if (sbase) step += (uint32_t)*sbase;  // device-resident step counter (graph-captured collect)
    const uint32_t gid = (uint32_t)(env_offset + n);
    const uint32_t a = (uint32_t)actions[n];
    const ppox::u32x4 ev = ppox::philox4x32_10(ppox::u32x4{EVENT_BLOCK, gid, step, a}, k0, k1);
    const float rew = ppox::u01(ev.x) < p_reward ? 1.f : 0.f;
    const bool done = ppox::u01(ev.y) < p_done;
    const uint4* s = reinterpret_cast<const uint4*>(in + n * 4LL * FRAME);
    uint4* o = reinterpret_cast<uint4*>(out + n * 4LL * FRAME);
    const uint4 z = make_uint4(0, 0, 0, 0);
    for (int c = threadIdx.x; c < CHUNKS; c += blockDim.x) {
        const ppox::u32x4 w = ppox::philox4x32_10(ppox::u32x4{(uint32_t)c, gid, step, a}, k0, k1);
        const uint4 f1 = done ? z : s[CHUNKS + c];
        const uint4 f2 = done ? z : s[2 * CHUNKS + c];
        const uint4 f3 = done ? z : s[3 * CHUNKS + c];
        o[c] = f1;
        o[CHUNKS + c] = f2;
        o[2 * CHUNKS + c] = f3;
        o[3 * CHUNKS + c] = make_uint4(w.x, w.y, w.z, w.w);
    }
    if (threadIdx.x == 0) {
        rewards[n] = rew;
        dones[n] = done ? 1 : 0;
        episode_update(ep, n, rew, done);
    }
}

// Low-dimensional Box-observation env (CartPole/MuJoCo-shaped): obs uniform in
// [-1, 1), reward 1 per step, done ~ Bernoulli(p_done) or at max_len.
__global__ void __launch_bounds__(256) vec_step_kernel(float* __restrict__ obs, const int32_t* __restrict__ actions,
                                                       long long N, int D, long long env_offset, uint32_t k0,
                                                       uint32_t k1, uint32_t step, float p_done, int max_len,
                                                       float* __restrict__ rewards, uint8_t* __restrict__ dones,
                                                       Episode ep, int reset) {
    const long long n = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (n >= N) return;
    const uint32_t gid = (uint32_t)(env_offset + n);
    const uint32_t a = reset ? RESET_ACTION : (actions ? (uint32_t)actions[n] : 0u);
    for (int b = 0; b * 4 < D; ++b) {
        const ppox::u32x4 w = ppox::philox4x32_10(ppox::u32x4{(uint32_t)b, gid, step, a}, k0, k1);
        const uint32_t ws[4] = {w.x, w.y, w.z, w.w};
        for (int j = 0; j < 4 && b * 4 + j < D; ++j) obs[n * D + b * 4 + j] = ppox::u01(ws[j]) * 2.f - 1.f;
    }
    if (reset) {
        if (ep.ep_ret) {
            ep.ep_ret[n] = 0.f;
            ep.ep_len[n] = 0;
        }
        return;
    }
    const ppox::u32x4 ev = ppox::philox4x32_10(ppox::u32x4{EVENT_BLOCK, gid, step, a}, k0, k1);
    const int len = ep.ep_len ? ep.ep_len[n] + 1 : 0;
    const bool done = ppox::u01(ev.y) < p_done || (max_len > 0 && len >= max_len);
    rewards[n] = 1.f;
    dones[n] = done ? 1 : 0;
    episode_update(ep, n, 1.f, done);
}

}  // namespace

extern "C" int ppox_atari_env_reset(uint8_t* obs, int64_t N, int64_t env_offset, uint64_t seed, float* ep_ret,
                                    int32_t* ep_len, void* stream) {
    PPOX_REQUIRE(obs && N > 0 && ppox::aligned16(obs), "ppox_atari_env_reset: bad arguments");
    Episode ep{ep_ret, ep_len, nullptr, nullptr};
    atari_reset_kernel<<<(unsigned)N, 256, 0, ppox::as_stream(stream)>>>(obs, env_offset, (uint32_t)seed,
                                                                         (uint32_t)(seed >> 32), ep);
    PPOX_LAUNCHED("ppox_atari_env_reset");
}

static int atari_env_step_impl(const uint8_t* obs_in, uint8_t* obs_out, const int32_t* actions, int64_t N,
                               int64_t env_offset, uint64_t seed, int64_t step, const int64_t* step_base,
                               float p_reward, float p_done, float* rewards, uint8_t* dones, float* ep_ret,
                               int32_t* ep_len, float* done_ret, int32_t* done_len, void* stream) {
    PPOX_REQUIRE(obs_in && obs_out && actions && rewards && dones && N > 0, "ppox_atari_env_step: null pointer");
    PPOX_REQUIRE(ppox::aligned16(obs_in) && ppox::aligned16(obs_out), "ppox_atari_env_step: obs must be 16B aligned");
    PPOX_REQUIRE(step_base || (step >= 1 && step < (1LL << 32)), "ppox_atari_env_step: step must be in [1, 2^32)");
    PPOX_REQUIRE((ep_ret == nullptr) == (ep_len == nullptr), "ppox_atari_env_step: ep_ret/ep_len pair");
    Episode ep{ep_ret, ep_len, done_ret, done_len};
    atari_step_kernel<<<(unsigned)N, 256, 0, ppox::as_stream(stream)>>>(
        obs_in, obs_out, actions, env_offset, (uint32_t)seed, (uint32_t)(seed >> 32), (uint32_t)step,
        reinterpret_cast<const long long*>(step_base), p_reward, p_done, rewards, dones, ep);
    PPOX_LAUNCHED("ppox_atari_env_step");
}

extern "C" int ppox_atari_env_step(const uint8_t* obs_in, uint8_t* obs_out, const int32_t* actions, int64_t N,
                                   int64_t env_offset, uint64_t seed, int64_t step, float p_reward, float p_done,
                                   float* rewards, uint8_t* dones, float* ep_ret, int32_t* ep_len, float* done_ret,
                                   int32_t* done_len, void* stream) {
    return atari_env_step_impl(obs_in, obs_out, actions, N, env_offset, seed, step, nullptr, p_reward, p_done, rewards,
                               dones, ep_ret, ep_len, done_ret, done_len, stream);
}

extern "C" int ppox_atari_env_step_dc(const uint8_t* obs_in, uint8_t* obs_out, const int32_t* actions, int64_t N,
                                      int64_t env_offset, uint64_t seed, const int64_t* step_base, int64_t step_off,
                                      float p_reward, float p_done, float* rewards, uint8_t* dones, float* ep_ret,
                                      int32_t* ep_len, float* done_ret, int32_t* done_len, void* stream) {
    PPOX_REQUIRE(step_base, "ppox_atari_env_step_dc: null step counter");
    return atari_env_step_impl(obs_in, obs_out, actions, N, env_offset, seed, step_off, step_base, p_reward, p_done,
                               rewards, dones, ep_ret, ep_len, done_ret, done_len, stream);
}

__global__ void counters_add_kernel(long long* c, int n, long long delta) {
    if ((int)threadIdx.x < n) c[threadIdx.x] += delta;
}

extern "C" int ppox_counters_add(int64_t* counters, int32_t n, int64_t delta, void* stream) {
    PPOX_REQUIRE(counters && n >= 1 && n <= 64, "ppox_counters_add: bad arguments");
    counters_add_kernel<<<1, 64, 0, ppox::as_stream(stream)>>>(reinterpret_cast<long long*>(counters), n, delta);
    PPOX_LAUNCHED("ppox_counters_add");
}

extern "C" int ppox_vec_env_reset(float* obs, int64_t N, int32_t D, int64_t env_offset, uint64_t seed, float* ep_ret,
                                  int32_t* ep_len, void* stream) {
    PPOX_REQUIRE(obs && N > 0 && D > 0, "ppox_vec_env_reset: bad arguments");
    Episode ep{ep_ret, ep_len, nullptr, nullptr};
    vec_step_kernel<<<ppox::ceil_div(N, 256), 256, 0, ppox::as_stream(stream)>>>(
        obs, nullptr, N, D, env_offset, (uint32_t)seed, (uint32_t)(seed >> 32), 0u, 0.f, 0, nullptr, nullptr, ep, 1);
    PPOX_LAUNCHED("ppox_vec_env_reset");
}

extern "C" int ppox_vec_env_step(float* obs, const int32_t* actions, int64_t N, int32_t D, int64_t env_offset,
                                 uint64_t seed, int64_t step, float p_done, int32_t max_len, float* rewards,
                                 uint8_t* dones, float* ep_ret, int32_t* ep_len, float* done_ret, int32_t* done_len,
                                 void* stream) {
    PPOX_REQUIRE(obs && rewards && dones && N > 0 && D > 0, "ppox_vec_env_step: bad arguments");
    PPOX_REQUIRE(step >= 1 && step < (1LL << 32), "ppox_vec_env_step: step must be in [1, 2^32)");
    Episode ep{ep_ret, ep_len, done_ret, done_len};
    vec_step_kernel<<<ppox::ceil_div(N, 256), 256, 0, ppox::as_stream(stream)>>>(
        obs, actions, N, D, env_offset, (uint32_t)seed, (uint32_t)(seed >> 32), (uint32_t)step, p_done, max_len,
        rewards, dones, ep, 0);
    PPOX_LAUNCHED("ppox_vec_env_step");
}
