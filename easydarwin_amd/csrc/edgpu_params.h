// edgpu_params.h -- kernel argument blocks (shared by edgpu_kernels.hip and edgpu_engine.cpp).
#pragma once
#include <stdint.h>
#include "edgpu.h"
#include "edgpu_device.h"

namespace edgpu {

struct IngestParams {
    const edgpu_pkt_desc* desc;
    const uint32_t* seg_off;
    const uint32_t* seg_sess;
    const uint8_t* blob;
    SessionDev* sessions;
    SenderDev* senders;
    StreamDev* streams;
    uint32_t* pflags;       // per desc: bit0 enqueued, bit1 video key, bit2 audio event, bits 8-15 local sender
    uint64_t* pidx;         // per desc: sender queue index
    CopyJob* jobs;          // per desc: slot copy for k_ingest_copy
    uint32_t npk;           // descriptors in the batch
    uint32_t copy_mode;     // 0: copy inside k_ingest, 1: k_ingest_copy (EDGPU_INGEST)
    uint32_t ablate;        // timing experiments only (EDGPU_ABLATE bits 4-7)
    uint32_t filter_ssrc;
    uint32_t ssrc_timeout_s;
    uint32_t overlap;       // check the ring against the in-flight fan-out window (fan_lo/fan_vlo)
    TickTotals* totals;
};

struct KeyframeParams {
    const uint32_t* seg_off;
    const uint32_t* seg_sess;
    const uint32_t* pflags;
    const uint64_t* pidx;
    SessionDev* sessions;
    SenderDev* senders;
};

struct PlanParams {
    SenderDev* senders;
    SubDev* subs;
    const uint32_t* sub_index;
    const uint32_t* sub_pos;    // SubDev index -> position in sub_index order (~0: inactive)
    const uint32_t* sub_range;  // per sender [begin, end) into sub_index
    edgpu_substream_out* sub_out;
    FanWork* work;
    FanSub* fansub;             // per sub_index position
    uint64_t* blk_bytes;        // per K2 block partials
    uint32_t* blk_count;
    uint64_t* blk_bytes_base;
    uint32_t* blk_count_base;
    TickTotals* totals;
    TickParams T;
};

struct FanoutParams {
    const SenderDev* senders;
    const uint32_t* sub_range;  // per sender [begin, end) into sub_index
    const SubDev* subs;
    const uint32_t* sub_index;
    const FanWork* work;
    const FanSub* fansub;
    uint8_t* arena;
    edgpu_out_desc* desc;
    uint64_t arena_words;       // capacities: stores outside them are dropped and flagged
    uint32_t max_desc;
    TickTotals* totals;
    uint32_t ablate;            // timing-only builds: bit0 skip descriptors, bit1 skip arena stores
};

struct ImageParams {
    SenderDev* senders;
    SessionDev* sessions;
    StreamDev* streams;
    ImgPlan* plan;
    uint32_t nplan;
    int64_t now;
    int64_t over_buffer_ms;
    uint8_t* buf;           // export: destination images; import: source images
    int* status;            // first error wins
};

}  // namespace edgpu
