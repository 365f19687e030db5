// The pre-RCCL presence check of st_comm_init (st_rendezvous.hip); internal.
#pragma once

#include <functional>

namespace st {

constexpr int kRdvIdBytes = 128;      // st_comm_unique_id's id
constexpr int kRdvPayloadBytes = 128; // what the host hands every rank (the RCCL id)

// A new rendezvous id (listener opened in this process, bound to the address
// it advertises: `addr`, dotted IPv4; NULL = ST_COMM_ADDR / the interface
// choice); 0 or -1.  A listener not joined within `ttl` seconds is closed by
// a later call.
int rdv_make_id(char* out, const char* addr, double ttl);

// Close the listener of an id this process made and has not joined: 0, or
// 1 if there is none (joined, released, or not made here); -1 on a foreign id.
int rdv_release(const char* id);

// Join the rendezvous of `id` as `rank` of `nranks`.  The first call in the
// process that made the id hosts it: once every rank is present it calls
// make_payload (ncclGetUniqueId) and hands the bytes to all.  Returns 0 with
// `payload` filled, or -1 (error set, naming missing ranks) after `limit` s.
int rdv_join(const char* id, int nranks, int rank, int device, double limit,
             const std::function<int(char*)>& make_payload, char* payload);

} // namespace st
