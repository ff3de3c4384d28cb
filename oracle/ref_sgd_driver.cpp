/*
 * ref_sgd_driver.cpp -- TEST INFRASTRUCTURE ONLY.
 *
 * extern "C" driver around the reference's own sparse SGD
 * (/root/reference/backend/src/optim/sgd.cpp, compiled in place by
 * oracle/Makefile into oracle/_ref/libstg_ref_sgd.so against the local torch
 * headers/libraries).  Drives SGD::configure (sgd.cpp:265-300) and
 * SGD::optimize_raw (sgd.cpp:34-263).
 */
#include <cstring>
#include <memory>
#include <mutex>
#include <string>
#include <unordered_map>
#include <torch/extension.h>
#include <torch/torch.h>

// expose the momentum map for read-back (all system headers already included)
#define private public
#include "optim/sgd.h"
#undef private

#define REF_API extern "C" __attribute__((visibility("default")))

REF_API void *ref_sgd_new(float lr, float momentum, float dampening, float weight_decay, int nesterov,
                          int maximize) {
    auto *o = new SGD();
    std::string k;
    o->set_lr(lr);
    k = "momentum"; o->configure(k, momentum);
    k = "dampening"; o->configure(k, dampening);
    k = "weight_decay"; o->configure(k, weight_decay);
    k = "nestrov"; o->configure(k, (bool)nesterov);
    k = "maximize"; o->configure(k, (bool)maximize);
    return o;
}
REF_API void ref_sgd_free(void *o) { delete static_cast<SGD *>(o); }
REF_API void ref_sgd_apply(void *o, const char *name, float *param, uint32_t param_len, float *g,
                           uint32_t *gidx, uint32_t glen) {
    static_cast<SGD *>(o)->optimize_raw(param, param_len, name, g, gidx, glen);
}
REF_API int ref_sgd_momentum(void *o, const char *name, float *out, uint32_t len) {
    auto *s = static_cast<SGD *>(o);
    auto it = s->m_optim_state_b.find(name);
    if (it == s->m_optim_state_b.end()) return -1;
    std::memcpy(out, it->second.get(), sizeof(float) * len);
    return 0;
}
