// Generations of the IPC exchange's interprocess events (pr_ipc.hip; ADVICE r5: shared with the CPU
// model checker host/ipc_model.cpp, so the rotation and the waiter's choice are model-checked).
// Plain C++, no HIP.
//
// The HIP runtime's interprocess events take at most 32 records each (profiles/r05/ipc_events/), so
// an owner records one event for at most kIpcRecordsPerEvent exchanges and then starts a fresh one
// (a new generation) in the next of kIpcGens page slots, stamped with the first exchange it serves
// and a generation id that only grows; a fresh generation also starts whenever the exchange counts
// restart (a new enable: `epoch`).  A waiter that needs exchange k takes the newest slot whose range
// [first_k, first_k + kIpcRecordsPerEvent) holds k.
#pragma once

#include <stdint.h>

namespace pr {

constexpr int64_t kIpcRecordsPerEvent = 30;  // below the runtime's 32-record ring
constexpr int kIpcGens = 3;                  // page slots per event

// The owner's view of one event: per slot the first exchange it serves; the current slot.
struct IpcGenOwner {
  int64_t first_k[kIpcGens] = {0, 0, 0};
  int64_t epoch = -1;  // of the current generation
  int cur = -1;        // -1: none yet
};

// The slot of a fresh generation for the owner's record of exchange k, or -1 when the current
// generation serves k.  The caller creates the event in that slot, publishes it and then calls
// ipc_gen_started.
inline int ipc_gen_rotate(const IpcGenOwner &o, int64_t k, int64_t epoch) {
  if (o.cur >= 0 && o.epoch == epoch && k >= o.first_k[o.cur] && k < o.first_k[o.cur] + kIpcRecordsPerEvent)
    return -1;
  return (o.cur + 1) % kIpcGens;
}
inline void ipc_gen_started(IpcGenOwner &o, int slot, int64_t k, int64_t epoch) {
  o.first_k[slot] = k;
  o.epoch = epoch;
  o.cur = slot;
}

// The waiter's choice for exchange k among a peer's slots (id 0: empty), or -1 if none holds k.
inline int ipc_gen_pick(const int64_t (&id)[kIpcGens], const int64_t (&first_k)[kIpcGens], int64_t k) {
  int best = -1;
  int64_t best_id = 0;
  for (int i = 0; i < kIpcGens; ++i)
    if (id[i] > best_id && first_k[i] <= k && k < first_k[i] + kIpcRecordsPerEvent) {
      best = i;
      best_id = id[i];
    }
  return best;
}

}  // namespace pr
