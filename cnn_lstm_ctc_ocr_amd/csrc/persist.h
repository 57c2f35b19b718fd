// Shared pieces of the persistent recurrent time loops (lstm_persistent.hip,
// gru_persistent.hip): the group/member placement, the XCD census that picks
// the hand-off form, the hand-off primitives and the bounded group wait.
//
// A "group" is one (direction, 32-row batch slice); its members are the
// workgroups that each own 32 hidden units. Per hand-off every member
// publishes its slice of a [32 x N] bf16 row block, drains its stores
// (vmcnt 0), barriers, and one lane raises the member's flag word; consumers
// poll all flags of the group, barrier, then load the rows. Form:
// MI355X_MICROARCH.md "Valid forms", row 1 (sc1 payload + sc1 flag, any
// placement); when the census finds the whole group on one XCD the traffic
// stays in that XCD's L2 (plain stores, nt loads).
#pragma once
#include <cstdlib>

#include "common.h"
#include "mfma_util.h"

namespace {

constexpr int PBR = 32, PHU = 32;          // batch rows, hidden units per workgroup
typedef __attribute__((address_space(1))) unsigned gu32;            // hand-off words: global, never flat
typedef __attribute__((address_space(1))) unsigned long long gu64;

__device__ __forceinline__ unsigned short bf16_bits(float x) {
    bf16 b = (bf16)x;
    return __builtin_bit_cast(unsigned short, b);
}
__device__ __forceinline__ float bits_f(unsigned short u) {
    return __uint_as_float((unsigned)u << 16);
}
__device__ __forceinline__ unsigned long long pack4(const float (&v)[4]) {
    return (unsigned long long)((unsigned)bf16_bits(v[0]) | ((unsigned)bf16_bits(v[1]) << 16)) |
           ((unsigned long long)((unsigned)bf16_bits(v[2]) | ((unsigned)bf16_bits(v[3]) << 16)) << 32);
}

// workgroup -> (group, member): members of a group share blockIdx % 8 when the
// grid allows it (speed only)
__device__ __forceinline__ void persistent_role(int ngroups, int nu, int& group, int& member) {
    const int id = blockIdx.x, grid = ngroups * nu;
    if (grid % 8 == 0 && (grid / 8) % nu == 0) {
        const int per = grid / 8, j = id / 8;
        group = (id % 8) * (per / nu) + j / nu;
        member = j % nu;
    } else {
        group = id / nu;
        member = id % nu;
    }
}

// Launch setup of a persistent recurrent kernel: the hand-off words count ON
// across launches, so the caller never clears them (no memset launch in front
// of every loop). flags[0, grid) are the members' flag words, flags[grid,
// 2 grid) their XCC census words (`grid` = gridDim.x). Every member of every
// group ends a launch at the same flag count, so a member's OWN flag, read at
// launch start, is this launch's base: the waits are for base + n. Census
// words carry a generation in bits 31:4 (the member's previous word + 1) and
// the XCC id + 1 in bits 3:0, so last launch's words never pass for this
// one's. A zeroed buffer is a valid start (base 0, generation 1).
//
// Are all members of this workgroup's group on ONE XCD? Each workgroup posts
// its HW_REG_XCC_ID (+1) once per launch (sc1), wave 0 waits for the group's
// posts and compares. Placement is the dispatcher's choice: it is measured
// here, never assumed. On one XCD the group's hand-offs stay in that XCD's L2
// (plain stores keep the lines in L2; nt loads bypass only the reader's L1);
// otherwise they use the placement-independent sc1 form.
__device__ __forceinline__ bool persistent_setup(gu32* flags, int group, int nu, int member, unsigned* err,
                                                 unsigned spin_limit, unsigned& base) {
    __shared__ unsigned s_setup[3];
    const int tid = threadIdx.x, lane = tid & 63;
    gu32* xtab = flags + gridDim.x + group * nu;
    if (tid == 0) {
        unsigned x;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(x));
        s_setup[0] = __hip_atomic_load(flags + group * nu + member, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const unsigned gen = (__hip_atomic_load(xtab + member, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >> 4) + 1u;
        s_setup[1] = gen;
        __hip_atomic_store(xtab + member, (gen << 4) | ((x & 15u) + 1u), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
    if (tid < 64) {
        const unsigned gen = s_setup[1];
        unsigned v = (gen << 4) | 1u, spins = 0;
        while (true) {
            if (lane < nu) v = __hip_atomic_load(xtab + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (__all((v >> 4) == gen)) break;
            __builtin_amdgcn_s_sleep(1);
            if (++spins > spin_limit) {
                if (lane == 0) __hip_atomic_fetch_or(err, (unsigned)OCRK_STATUS_LSTM_CENSUS, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                break;
            }
        }
        const unsigned first = __shfl(v & 15u, 0, 64);
        const bool same = __all(lane >= nu || ((v >> 4) == gen && (v & 15u) == first));
        if (lane == 0) s_setup[2] = same ? 1u : 0u;
    }
    __syncthreads();
    base = s_setup[0];
    return s_setup[2] != 0;
}

// pause between hand-off polls (s_sleep units of 64 clocks; OCRK_POLL_SLEEP at build time, 0 = spin)
#ifndef OCRK_POLL_SLEEP
#define OCRK_POLL_SLEEP 1
#endif
__device__ __forceinline__ void poll_pause() {
    if constexpr (OCRK_POLL_SLEEP > 0) __builtin_amdgcn_s_sleep(OCRK_POLL_SLEEP);
}

// wrap-safe "count has reached target" for the counting flag words
__device__ __forceinline__ bool reached(unsigned count, unsigned target) { return (int)(count - target) >= 0; }

// The two hand-off forms (see group_on_one_xcd): flag poll, flag raise,
// 8-B payload store, 16-B payload load.
__device__ __forceinline__ unsigned poll_word(gu32* p, bool local) {
    if (local) {
        asm volatile("" ::: "memory");
        return __builtin_nontemporal_load(p);
    }
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void raise_flag(gu32* p, unsigned v, bool local) {
    if (local) *p = v;
    else __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void put8(gu64* p, unsigned long long v, bool local) {
    if (local) *p = v;
    else __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ ocrk::u32x4 get16(__amdgpu_buffer_rsrc_t r, int off, bool local) {
    return local ? __builtin_bit_cast(ocrk::u32x4, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 2))     // nt
                 : __builtin_bit_cast(ocrk::u32x4, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 16));   // sc1
}

// Wave 0 waits until every member flag of the group is >= target, then the
// workgroup barriers. Bounded: past spin_limit polls it ORs `bit` into the
// status word and marks the loop dead (*dead, wave-0 register), so later
// waits return at once and the kernel runs to completion (results garbage,
// reported through the status word -- never a hang).
__device__ __forceinline__ void group_wait(gu32* gflags, int nu, unsigned target, bool local, unsigned* err,
                                           unsigned bit, unsigned spin_limit, bool& dead) {
    if (threadIdx.x < 64 && !dead) {
        const int lane = threadIdx.x;
        unsigned spins = 0;
        while (true) {
            unsigned f = target;
            if (lane < nu) f = poll_word(gflags + lane, local);
            if (__all(reached(f, target))) break;
            poll_pause();
            if (++spins > spin_limit) {
                if (lane == 0) __hip_atomic_fetch_or(err, bit, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                dead = true;
                break;
            }
        }
    }
    __syncthreads();
}

// Publish done: drain this thread's payload stores, barrier, one lane raises the flag.
__device__ __forceinline__ void group_post(gu32* flag, unsigned v, bool local) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) raise_flag(flag, v, local);
}

// polls before a hand-off wait gives up: option LSTM_SPIN_LIMIT (tests force tiny
// limits; it bounds every persistent recurrence), default 1 << 22
inline unsigned recur_spin_limit() {
    const int64_t v = ocrk::opt(ocrk::OPT_LSTM_SPIN_LIMIT);
    return v > 0 && v < (1ll << 32) ? (unsigned)v : (1u << 22);
}

// flag word + XCC word per workgroup, rounded to a 128-B block (the size of a
// caller-kept counting buffer as well: ocrk_persistent_flags_size)
inline size_t persistent_counter_bytes(int B, int H) {
    return ((size_t)2 * 2 * (B / PBR) * (H / PHU) * sizeof(unsigned) + 127) / 128 * 128;
}

}  // namespace
