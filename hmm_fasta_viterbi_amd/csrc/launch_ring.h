// launch_ring.h -- launch slots of one device profile (host side), shared by the MSV profile
// (msv_device.cpp) and the Viterbi profile (vit_device.cpp).
//
// A persistent kernel takes its work from a device counter pair {next index, waves left} that its last
// wave puts back to zero.  Two launches of one profile that overlap on different streams must not
// share a pair (sequences would be skipped or scored twice), so every launch takes the next of N
// slots, and a slot is reused only after its previous launch: nothing to do on the same stream, an
// event wait when the streams differ.  An event record is a packet on the stream (~4 us between a
// launch and the next one, 3% of a 0.14 ms cfg2 kernel), so it is recorded lazily -- only when another
// stream wants the slot -- for streams known to outlive that moment (the library's own streams and a
// caller stream bound to the profile); a launch on any other caller stream records its event at once
// (that stream may be destroyed before the next launch).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace msvrt {

template <int N>
struct LaunchRing {
    hipEvent_t done[N] = {};
    hipStream_t last[N] = {};  // nullptr: never launched
    bool recorded[N] = {};     // done[k] covers the slot's last launch
    bool dirty[N] = {};        // a launch failed after the slot's counters were touched
    uint32_t next = 0;

    // Creates every slot's event up front (created lazily, the first N launches of a fresh profile
    // would each pay an event creation).
    hipError_t create_events() {
        for (hipEvent_t& e : done)
            if (!e) {
                // device-scope release: the event only orders this device's streams
                const hipError_t r = hipEventCreateWithFlags(&e, hipEventDisableTiming | hipEventReleaseToDevice);
                if (r != hipSuccess) return r;
            }
        return hipSuccess;
    }

    // Takes the next slot for a launch on `st`; makes `st` wait for the slot's previous launch if
    // that ran on another stream.
    hipError_t acquire(hipStream_t st, int* slot) {
        const int k = static_cast<int>(next++ % N);
        if (!done[k]) {
            const hipError_t e = hipEventCreateWithFlags(&done[k], hipEventDisableTiming | hipEventReleaseToDevice);
            if (e != hipSuccess) return e;
        }
        if (last[k] && last[k] != st) {
            // Nothing to wait for when the slot's last launch has completed: its stream is idle, or its
            // recorded event has fired (host queries, no packets -- a fused grid call acquires a slot
            // of every profile, and 24 record + wait pairs cost ~0.3 ms before the launch).
            const bool finished = recorded[k] ? hipEventQuery(done[k]) == hipSuccess
                                              : hipStreamQuery(last[k]) == hipSuccess;
            if (!finished) {
                if (!recorded[k]) {  // lazy: last[k] is a live stream; this covers all of its work so far
                    const hipError_t e = hipEventRecord(done[k], last[k]);
                    if (e != hipSuccess) return e;
                    recorded[k] = true;
                }
                const hipError_t e = hipStreamWaitEvent(st, done[k], 0);
                if (e != hipSuccess) return e;
            }
            (void)hipGetLastError();  // a query's hipErrorNotReady is not an error
        }
        *slot = k;
        return hipSuccess;
    }
    // `lazy`: `st` is known to stay alive until the next acquire of this slot or flush()
    hipError_t release(int k, hipStream_t st, bool lazy) {
        last[k] = st;
        recorded[k] = !lazy;
        return lazy ? hipSuccess : hipEventRecord(done[k], st);
    }
    // Records the pending lazy events of stream `st` (before it stops being guaranteed alive).
    hipError_t flush(hipStream_t st) {
        for (int k = 0; k < N; ++k)
            if (last[k] == st && !recorded[k]) {
                const hipError_t e = hipEventRecord(done[k], st);
                if (e != hipSuccess) return e;
                recorded[k] = true;
            }
        return hipSuccess;
    }
    void destroy() {
        for (hipEvent_t& e : done)
            if (e) (void)hipEventDestroy(e);
    }
};

}  // namespace msvrt
