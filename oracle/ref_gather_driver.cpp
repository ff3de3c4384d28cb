/*
 * ref_gather_driver.cpp -- TEST INFRASTRUCTURE ONLY.
 *
 * extern "C" driver around the reference's own add_arrays
 * (/root/reference/backend/src/misc/array_util.h:12-54, included in place by
 * oracle/Makefile into oracle/_ref/libstg_ref_gather.so with the reference
 * flags).  The per-rank loop of ModuleCpuGather::run (engine/modules/
 * cpu_gather.cpp:59-87) lives in an engine module that needs the whole engine
 * (torch, shm, zmq) to build, so its few lines of control flow are restated
 * here around the reference's arithmetic: slice [len*r/N, len*(r+1)/N) of
 * grad[0] += residual, then += grad[1], ..., += grad[N-1].
 */
#include <cstddef>
#include <cstdint>
#include "misc/array_util.h"

#define REF_API extern "C" __attribute__((visibility("default")))

REF_API void ref_gather_add(float *grad0, const float *resid, const float *const *grads, int num_gpus,
                            int64_t len, int local_rank) {
    const int64_t start = (len * local_rank) / num_gpus, end = (len * (local_rank + 1)) / num_gpus;
    for (int i = 0; i < num_gpus; ++i) {
        const float *src = (i == 0 ? resid : grads[i]) + start;
        add_arrays(grad0 + start, src, (size_t)(end - start));
    }
}
