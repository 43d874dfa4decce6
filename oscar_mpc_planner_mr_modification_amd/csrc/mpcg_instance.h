// mpcg_instance.h — compiled kernel instances of the batched SQP solve.
//
// The kernel is specialised at compile time on the generated solver's dimensions, as
// the reference's acados / Forces solvers are generated per configuration
// (solver_generator/generate_solver.py).  An instance is one Cfg<N, n_lin, n_ell,
// n_scen, nx, model>; it registers its launcher with libmpcg.so's instance table from a
// static initialiser, so a translation unit with MPCG_DEFINE_INSTANCE(...) adds a
// shape to any process that loads it: the built-in instances (mpcg_inst_*.hip in
// libmpcg.so) and the one codegen.py writes for a generated solver directory
// (mpcg_instance.hip, compiled into the drop-in libmpc_planner_solver.so).
#pragma once
#include <hip/hip_runtime.h>

#include <atomic>
#include <cstdio>

#include "mpcg.h"
#include "mpcg_sqp.h"

extern "C" {
/* launcher of one compiled instance: enqueues the solve of `batch` problems on `stream`
 * and returns the hipError_t of the launch.  `workspace`: device memory on the stream's device
 * of at least MPCG_QUEUE_BYTES + batch x the instance's workspace bytes per solve: the work
 * queue of sqp_kernel (zeroed on the stream before every launch), then per solve the stage
 * blocks of the instances whose blocks do not fit the LDS budget and the interior point's
 * iterative-refinement scratch */
typedef int (*mpcg_instance_launch)(const mpcg_problem* pr, int batch, const mpcg_io* io, void* stream,
                                    unsigned long long* stamps, void* workspace);
/* libmpcg.so's instance table: (model, N, n_lin, n_ell, n_scen, nx) -> launcher, the
 * doubles of one solve's QP memory and the workspace bytes of one solve.  Returns 0 (a
 * shape already present keeps its first launcher); -3, and the instance stays unknown,
 * when `abi_version` is not libmpcg.so's MPCG_ABI_VERSION (an instance library compiled
 * against other sources: mpcg_rejected_instances() counts them). */
int mpcg_register_instance(int abi_version, int model, int N, int n_lin, int n_ell, int n_scen, int nx, mpcg_instance_launch fn,
                           int qp_mem_size, long long workspace_bytes_per_solve, const char* traits);
/* instance registrations refused for another ABI since libmpcg.so loaded */
int mpcg_rejected_instances(void);
}
/* the work-queue words at the head of an instance workspace (sqp_kernel) */
#define MPCG_QUEUE_BYTES 256

namespace mpcg {

// grid of a work-queue launch: the workgroups the stream's device holds at once (occupancy x
// CUs), at most one per problem; cached per device.  MPCG_QUEUE_GRID_PER_CU (A/B only) sets the
// workgroups per CU.
template <class C, bool FULL, int PROF, int MODE = MODE_FUSED>
int queue_grid(int batch, hipStream_t stream) {
    constexpr int MAXDEV = 64;
    static std::atomic<int> resident[MAXDEV];  // 0: not yet asked, -1: no answer
    int dev = 0;
    if ((stream ? hipStreamGetDevice(stream, &dev) : hipGetDevice(&dev)) != hipSuccess || dev < 0 || dev >= MAXDEV)
        return batch;
    int r = resident[dev].load(std::memory_order_relaxed);
    if (r == 0) {
        int cus = 0, per_cu = 0;
        r = -1;
        if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && cus > 0) {
#ifdef MPCG_QUEUE_GRID_PER_CU
            per_cu = MPCG_QUEUE_GRID_PER_CU;
#else
            int cur = 0;
            const bool sw = hipGetDevice(&cur) == hipSuccess && cur != dev && hipSetDevice(dev) == hipSuccess;
            if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, sqp_kernel<C, FULL, PROF, MODE>, 64, 0) != hipSuccess)
                per_cu = 0;
            if (sw) (void)hipSetDevice(cur);
#endif
            if (per_cu > 0) r = per_cu * cus;
        }
        resident[dev].store(r, std::memory_order_relaxed);
    }
    // (no occupancy answer: one workgroup per problem, still through the queue)
    return r > 0 && r < batch ? r : batch;
}

template <class C, bool FULL, int PROF, int MODE = MODE_FUSED>
void launch_kernel(const mpcg_problem* pr, int batch, const mpcg_io* io, hipStream_t st, unsigned long long* stamps,
                   double* gws, unsigned* queue, int split_it = 0) {
    hipLaunchKernelGGL((sqp_kernel<C, FULL, PROF, MODE>), dim3(queue ? queue_grid<C, FULL, PROF, MODE>(batch, st) : batch),
                       dim3(64), 0, st, *pr, batch, *io, stamps, gws, queue, split_it);
}

// the split launch (split_on, MPCG_SPLIT): per RTI iteration a linearisation launch, then an interior-point
// launch, each zeroing its queue words first when it takes the work queue
template <class C, int PROF>
int launch_split(const mpcg_problem* pr, int batch, const mpcg_io* io, hipStream_t st, unsigned long long* stamps,
                 double* gws, unsigned* qw) {
#ifdef MPCG_SPLIT_WORDS
    // (diagnostic: one memset, a queue word of its own per launch)
    if (hipMemsetAsync(qw, 0, MPCG_QUEUE_BYTES, st) != hipSuccess) return (int)hipGetLastError();
#endif
    for (int it = 0; it < pr->sqp_iters; ++it) {
#ifdef MPCG_SPLIT_WORDS
        unsigned* ql = kernel_queue<C, MODE_LIN>() ? qw + (2 * it) % 64 : nullptr;
        unsigned* qq = kernel_queue<C, MODE_QP>() ? qw + (2 * it + 1) % 64 : nullptr;
#else
        unsigned* ql = kernel_queue<C, MODE_LIN>() ? qw : nullptr;
        unsigned* qq = kernel_queue<C, MODE_QP>() ? qw : nullptr;
        if (ql && hipMemsetAsync(ql, 0, MPCG_QUEUE_BYTES, st) != hipSuccess) return (int)hipGetLastError();
#endif
        launch_kernel<C, false, PROF, MODE_LIN>(pr, batch, io, st, stamps, gws, ql, it);
#ifdef MPCG_SPLIT_SYNC
        (void)hipStreamSynchronize(st);
#endif
#ifndef MPCG_SPLIT_WORDS
        if (qq && hipMemsetAsync(qq, 0, MPCG_QUEUE_BYTES, st) != hipSuccess) return (int)hipGetLastError();
#endif
        launch_kernel<C, false, PROF, MODE_QP>(pr, batch, io, st, stamps, gws, qq, it);
#ifdef MPCG_SPLIT_SYNC
        (void)hipStreamSynchronize(st);
#endif
    }
    return (int)hipGetLastError();
}

template <class C>
int launch_instance(const mpcg_problem* pr, int batch, const mpcg_io* io, void* stream, unsigned long long* stamps,
                    void* workspace) {
    // exactly one wavefront per workgroup: the kernel's lane exchanges rely on it (wave_sync).
    // The workspace (MPCG_QUEUE_BYTES + batch x the instance's bytes per solve) is required where it
    // is read: the GFH stage blocks, and the refinement scratch when the profile refines
    // (qp_itref_corr_max > 0, HPIPM's profile); a robust-profile call of an instance without GFH may
    // pass NULL (one workgroup per problem then, without the work queue)
    if ((gfh_doubles<C>() > 0 || split_on<C>() || (pr->qp_itref_corr_max > 0 && itref_doubles<C>() > 0)) &&
        !workspace)
        return (int)hipErrorInvalidValue;
    unsigned* queue = C::QUEUE && workspace ? (unsigned*)workspace : nullptr;
    double* gws = workspace ? (double*)((char*)workspace + MPCG_QUEUE_BYTES) : nullptr;
    const hipStream_t st = (hipStream_t)stream;
    // the queue counter starts at zero for every launch, whatever an earlier launch on this
    // workspace left behind (one that died mid-way included): a 256-byte memset on the stream
    if (queue && hipMemsetAsync(queue, 0, MPCG_QUEUE_BYTES, st) != hipSuccess) return (int)hipGetLastError();
    // the full variant only when the call needs QP memory, the warm start, the residuals or the full
    // SQP; the lean one specialised on the call's interior-point profile (qp_profile_kind), and a lean
    // call whose switches match neither profile on the full variant's run-time switches (without QP
    // memory, residuals or warm start the full variant runs the lean variant's operations)
    const int prof = qp_profile_kind(*pr);
    const bool full = io->stats || io->qp_in || io->qp_out || needs_full(*pr) || prof == PROF_RUNTIME;
    if constexpr (split_on<C>()) {
        if (!full && pr->sqp_iters > 0) {
            unsigned* qw = (unsigned*)workspace;
            return prof == PROF_HPIPM ? launch_split<C, PROF_HPIPM>(pr, batch, io, st, stamps, gws, qw)
                                      : launch_split<C, PROF_ROBUST>(pr, batch, io, st, stamps, gws, qw);
        }
    }
    if (full)
        launch_kernel<C, true, PROF_RUNTIME>(pr, batch, io, st, stamps, gws, queue);
    else if (prof == PROF_HPIPM)
        launch_kernel<C, false, PROF_HPIPM>(pr, batch, io, st, stamps, gws, queue);
    else
        launch_kernel<C, false, PROF_ROBUST>(pr, batch, io, st, stamps, gws, queue);
    return (int)hipGetLastError();
}

// the storage choices of an instance (mpcg_instance_traits): lane parts per stage, row slots
// per lane, stored 1/t, LEAN / GFH storage, constant [B A] rows, paired chains, LDS bytes, the
// stage strides (doubles) of the h-row gradients, the h-row gaps and the cost-to-go rows
template <class C>
const char* instance_traits() {
    static char buf[192];
    using L = LdsOf<C>;
    snprintf(buf, sizeof buf,
             "parts=%d slots=%d store_it=%d lean=%d gfh=%d fconst=%d pair=%d lds=%d strides=%d,%d,%d", C::PARTS,
             C::SLOTS, (int)C::STORE_IT, (int)lds_lean<C>(), (int)lds_gfh<C>(), (int)C::FCONST, (int)C::PAIR_CHAINS,
             (int)sizeof(L), L::DGS, L::HDS, L::PS);
    return buf;
}

template <class C>
int register_instance() {
    return mpcg_register_instance(MPCG_ABI_VERSION, C::MODEL, C::N, C::NL, C::NE, C::NS, C::NX, &launch_instance<C>, C::QPM,
                                  (long long)(ws_doubles<C>() * sizeof(double)), instance_traits<C>());
}

}  // namespace mpcg

#define MPCG_INST_CAT2(a, b) a##b
#define MPCG_INST_CAT(a, b) MPCG_INST_CAT2(a, b)
// one instance: Cfg<N, n_lin, n_ell, n_scen, nx, model>
#define MPCG_DEFINE_INSTANCE(N_, L_, E_, S_, X_, M_)                                                  \
    static const int MPCG_INST_CAT(mpcg_instance_reg_, __COUNTER__) =                                \
        mpcg::register_instance<mpcg::Cfg<N_, L_, E_, S_, X_, M_>>();
