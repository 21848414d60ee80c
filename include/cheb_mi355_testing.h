/* Test hooks of libcheb_mi355 -- NOT part of the integration surface
 * (include/cheb_mi355.h is).  They exist so the library's own tests can
 * provoke failure paths that a healthy GPU never takes; a caller of the
 * drop-in path never needs them.  Same ABI conventions as cheb_mi355.h.
 */
#ifndef CHEB_MI355_TESTING_H
#define CHEB_MI355_TESTING_H

#include "cheb_mi355.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Failure-detection test hook of the one-launch gconv-LSTM layer forward
 * (cg_lstm_seq_forward[_x]): from time step `step` on, workgroup 0 of pair 0
 * of this plan's sequence launches stops publishing its step counter, so its
 * partner times out exactly as when it is not co-resident: the launch poisons
 * the outputs it owed with NaN and sets the plan's fault word
 * (cg_lstm_seq_fault).  -1 (the default) is off.  Plan-scoped; nothing else
 * reads it.  Used by tests/test_gpu_lstm.py::test_seq_handoff_timeout_raises_and_poisons. */
int cg_plan_set_seq_fault_test(cg_plan* plan, int32_t step);

#ifdef __cplusplus
}
#endif

#endif /* CHEB_MI355_TESTING_H */
