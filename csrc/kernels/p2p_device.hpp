// Device-initiated point-to-point transport (p2p_device.hip): DAG edges moved by kernels on the
// ranks' own streams, so a step with cross-GPU edges captures into ONE hipGraph per rank.
//
// Protocol per edge (producer P -> consumer C, one slot per edge, values = the step number):
//   P, in stream order after the producing kernel:   ready[slot]@C  = step      (notify)
//   C, at the consumer:  wait ready[slot] >= step, copy P's region -> C's region (pull, over
//                        xGMI when P is another GPU), then ack[slot]@P = step
//   P, before overwriting the sent region again:     wait ack[slot] >= step    (wait)
// Every rank bumps its own step counter at the start of a step (tick), so the same captured
// graph replays with fresh sequence numbers. A wait that does not see its flag within the
// timeout sets an error word and gives up (wrong data, never a hung GPU); the host checks it.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

void launch_p2p_tick(int64_t* step, hipStream_t s);
void launch_p2p_notify(int64_t* remote_flag, const int64_t* step, hipStream_t s);
// dst <- src (bytes % 16 == 0, both 16-B aligned) once *ready >= *step; then ack_remote = step.
// `ticket` counts arriving workgroups (monotonic; its launches always use the same grid).
// `moved` (optional): a device byte counter of what the rank pulled (reports, tests)
void launch_p2p_pull(const void* src, void* dst, int64_t bytes, const int64_t* ready, int64_t* ack_remote,
                     unsigned* ticket, const int64_t* step, int* err, int64_t timeout_ticks, int blocks,
                     unsigned long long* moved, hipStream_t s);
// Routed-row pull (expert parallelism): rows [off[e], off[e+1]) of each listed expert, gathered
// through idx (hidden state -> expert GPU) or as compact rows (expert output -> combine); see
// p2p_device.hip. max_rows sizes the grid (the device-side counts decide what moves).
void launch_p2p_pull_rows(const void* src, void* dst, int64_t row_bytes, const int32_t* idx, const int32_t* off,
                          const int32_t* experts, int n_exp, int64_t max_rows, const int64_t* ready,
                          int64_t* ack_remote, unsigned* ticket, const int64_t* step, int* err, int64_t timeout_ticks,
                          unsigned long long* moved, hipStream_t s);
void launch_p2p_wait(const int64_t* flag, const int64_t* step, int* err, int64_t timeout_ticks, int code,
                     hipStream_t s);
int p2p_pull_blocks(int64_t bytes);

// The sends posted at one program point notify their consumers from ONE launch (up to
// kP2PBatch flags; a notify never waits). Pulls are not batched: a pull of one edge must not wait
// for another edge's flag before it acks (parallel/validate.py device_deadlock_check, batched).
constexpr int kP2PBatch = 16;
void launch_p2p_notify_many(int64_t* const* flags, int n, const int64_t* step, hipStream_t s);
