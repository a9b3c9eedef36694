// argmin_common.h -- the np.argmin result record (controllers.py:82-85), shared by the
// two-launch argmin (rollout.hip) and the split kernel's fused tail (rollout_x3.hip).
#pragma once
#include "device_common.h"
#include "kernels.h"

namespace bcmpc {

// Writes out->{best_index, best_cost, first_action} for the winning (cost, index) record
// (maximize: the record holds -cost).  CEM merge: np.argmin over the iteration-major
// concatenation keeps the earlier best on ties.
__device__ __forceinline__ void argmin_record(const ArgminArgs& a, Best best) {
    bcmpc_result* out = a.out;
    if (a.merge) {
        const double prev = out->best_cost;
        const Best ex{a.maximize ? -prev : prev, out->best_index - a.pos_base};
        if (!better(best, ex)) return;
    }
    out->best_index = (a.merge || a.cem_mu ? a.pos_base : a.cand_offset) + best.i;
    out->best_cost = a.maximize ? -best.c : best.c;
    for (int j = 0; j < BCMPC_MAX_ACTION; ++j) out->first_action[j] = 0.0;
    if (best.i < a.K) {
        const uint64_t g = (uint64_t)(a.cand_offset + best.i);
        for (int j = 0; j < a.A; ++j) {
            const double lo = a.consts[6 * 32 + j], hi = a.consts[7 * 32 + j];
            out->first_action[j] =
                a.act_out ? a.act_out[best.i * a.A + j]     // policy-mixed actions (controllers.py:233-235)
                : a.cem_mu ? cem_action(a.seed, g, 0, j, a.cem_iter, a.cem_mu[j], a.cem_sigma[j], lo, hi)
                : a.actions ? a.actions[best.i * a.A + j]   // action_paths[0, i*, :] (controllers.py:84-85)
                          : rng_action(a.seed, g, 0, j, lo, hi);
        }
    }
}

// the record, then (synchronous steps) the mapped done word: the host spins on it (capi.cpp
// wait_done) and reads the record after it sees seq
__device__ __forceinline__ void argmin_write(const ArgminArgs& a, Best best) {
    argmin_record(a, best);
    if (a.done) {
        __threadfence_system();
        __hip_atomic_store(a.done, a.seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

// The same record written by a whole block (best valid in thread 0; sc / si: >= 1 LDS slot): thread 0
// applies the merge rule and writes index and cost, threads j < BCMPC_MAX_ACTION write first_action[j] in
// parallel (the regenerated Philox / CEM actions are ~100 instructions each: one thread doing all A of
// them was most of a small-K argmin launch), then thread 0 raises the done word.
__device__ __forceinline__ void argmin_write_block(const ArgminArgs& a, Best best, double* sc, int64_t* si) {
    bcmpc_result* out = a.out;
    if (threadIdx.x == 0) {
        bool write = true;
        if (a.merge) {
            const double prev = out->best_cost;
            const Best ex{a.maximize ? -prev : prev, out->best_index - a.pos_base};
            write = better(best, ex);
        }
        si[0] = write ? best.i : -1;
        if (write) {
            out->best_index = (a.merge || a.cem_mu ? a.pos_base : a.cand_offset) + best.i;
            out->best_cost = a.maximize ? -best.c : best.c;
        }
    }
    __syncthreads();
    const int64_t bi = si[0];
    const int j = threadIdx.x;
    if (bi >= 0 && j < BCMPC_MAX_ACTION) {
        double v = 0.0;
        if (bi < a.K && j < a.A) {
            const uint64_t g = (uint64_t)(a.cand_offset + bi);
            const double lo = a.consts[6 * 32 + j], hi = a.consts[7 * 32 + j];
            v = a.act_out ? a.act_out[bi * a.A + j]
                : a.cem_mu ? cem_action(a.seed, g, 0, j, a.cem_iter, a.cem_mu[j], a.cem_sigma[j], lo, hi)
                : a.actions ? a.actions[bi * a.A + j]
                          : rng_action(a.seed, g, 0, j, lo, hi);
        }
        out->first_action[j] = v;
    }
    if (a.done) {
        __syncthreads();
        if (threadIdx.x == 0) {
            __threadfence_system();
            __hip_atomic_store(a.done, a.seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
    }
}

}  // namespace bcmpc
