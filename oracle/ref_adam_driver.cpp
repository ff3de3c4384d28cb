/*
 * ref_adam_driver.cpp -- TEST INFRASTRUCTURE ONLY.
 *
 * extern "C" driver around the reference's own sparse Adam
 * (/root/reference/backend/src/optim/adam.cpp, compiled in place by
 * oracle/Makefile into oracle/_ref/libstg_ref_adam.so against the local torch
 * headers/libraries).  Drives Adam::configure (adam.cpp:90-122) and
 * Adam::optimize_raw (adam.cpp:19-86); reads back the per-name state maps
 * (adam.h:16-19) so the goldens pin m, v, vmax and tick as well as param.
 */
#include <cstring>
#include <memory>
#include <mutex>
#include <string>
#include <unordered_map>
#include <torch/extension.h>
#include <torch/torch.h>

// expose the state maps for read-back (all system headers already included)
#define private public
#include "optim/adam.h"
#undef private

#define REF_API extern "C" __attribute__((visibility("default")))

REF_API void *ref_adam_new(float lr, float b1, float b2, float eps, float weight_decay, int amsgrad, int maximize) {
    auto *o = new Adam();
    std::string k;
    o->set_lr(lr);
    k = "b1"; o->configure(k, b1);
    k = "b2"; o->configure(k, b2);
    k = "eps"; o->configure(k, eps);
    k = "weight_decay"; o->configure(k, weight_decay);
    k = "amsgrad"; o->configure(k, (bool)amsgrad);
    k = "maximize"; o->configure(k, (bool)maximize);
    return o;
}
REF_API void ref_adam_free(void *o) { delete static_cast<Adam *>(o); }
REF_API void ref_adam_apply(void *o, const char *name, float *param, uint32_t param_len, float *g, uint32_t *gidx,
                            uint32_t glen) {
    static_cast<Adam *>(o)->optimize_raw(param, param_len, name, g, gidx, glen);
}
// m, v: param_len floats each; returns the tick the next call will use, -1 if the name is unknown
REF_API int ref_adam_state(void *o, const char *name, float *m, float *v, uint32_t len, float *vmax) {
    auto *s = static_cast<Adam *>(o);
    auto it = s->m_optim_state_m.find(name);
    if (it == s->m_optim_state_m.end()) return -1;
    std::memcpy(m, it->second.get(), sizeof(float) * len);
    std::memcpy(v, s->m_optim_state_v[name].get(), sizeof(float) * len);
    *vmax = s->m_optim_state_vmax[name];
    return (int)s->m_optim_state_tick[name];
}
