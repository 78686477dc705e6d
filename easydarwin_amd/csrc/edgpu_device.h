// edgpu_device.h -- device-resident tables of the relay engine (shared by host and kernels).
//
// HBM layout (one context = one GPU):
//   * per sender (track x {RTP socket, RTCP socket}, the reference's ReflectorSender,
//     ReflectorStream.h:274-351) two rings:
//       - a packet-metadata ring of PktMeta (32 B), power-of-two entries, indexed by the
//         sender's monotonically increasing packet index (its queue position);
//       - a byte ring of 16-B "slots": each packet occupies roundup16(4 + len) bytes,
//         [4-B RTSP-interleaved header '$' 0 BE16(len)][packet bytes][pad].  Slot offsets are
//         kept in a *virtual* byte space (vbyte, monotonic u64); the ring position is
//         vbyte mod ring_bytes, so a 16-B word never straddles the ring end.
//     The slot layout is also the fan-out output layout, so relaying a range of packets to a
//     subscriber is one contiguous, 16-B-aligned copy (UDP datagram at slot+4; TCP frame at
//     slot+0 with the channel byte patched).
//   * SenderDev / StreamDev / SessionDev / SubDev tables (AoS, small).
#pragma once
#include <stdint.h>

namespace edgpu {

enum : uint32_t {
    kMaxPacket = 2060,              // ReflectorPacket::kMaxReflectorPacketSize (ReflectorStream.h:126)
    kSlotWordsMax = 129,            // roundup16(4 + 2060) / 16: 16-B words of the largest slot
    kIngestThreads = 256,
    kMaxTracks = 16,                // per session
    kMaxSendersPerSession = 2 * kMaxTracks,
};

// SenderDev.flags
enum : uint32_t {
    kSndRtcpPort = 1u << 0,         // RTCP by local-port parity (bound UDP push socket B)
    kSndRtcpKind = 1u << 1,         // written with qtssWriteFlagsIsRTCP (second sender of a stream)
    kSndVideo    = 1u << 2,         // stream payload type video
    kSndH264     = 1u << 3,         // payload name exactly "H264/90000"
    kSndAudio    = 1u << 4,         // stream payload type audio
};

struct PktMeta {                    // 32 B
    uint64_t vbyte;                 // virtual offset of the packet's slot
    uint64_t id;                    // fStreamCountID
    int64_t  arrival;               // fTimeArrived
    uint16_t len;                   // fPacketPtr.Len (0 = rejected by the SSRC filter), <= 2060
    uint16_t seq;                   // GetPacketRTPSeqNum (ReflectorStream.h:180-189): 0 if len < 4
    uint32_t vcount;                // number of non-empty packets before this one (mod 2^32)
};

struct CopyJob {                    // 32 B: one enqueued packet's slot copy, blob -> byte ring
    uint64_t ring;                  // device pointer of the sender's byte ring (16-B words)
    uint64_t vword;                 // virtual word index of the slot
    uint32_t wmask;                 // ring words - 1
    uint32_t src_slot;              // slot index in the batch blob
    uint32_t len;                   // packet length (0: nothing to copy)
    uint32_t sender;                // global sender index (its vbyte_end bounds the live words)
};

struct SenderDev {
    // static
    uint64_t meta;                  // device pointer to PktMeta[ring_packets]
    uint64_t ring;                  // device pointer to the byte ring
    uint32_t pk_mask;               // ring_packets - 1
    uint32_t word_mask;             // ring_bytes / 16 - 1
    uint32_t flags;
    uint32_t session;
    uint32_t stream;                // global stream (track) index
    uint32_t track;
    uint64_t floor;                 // oldest index this sender ever held (> 0 only for a
                                    // replica session built from a session image)
    // dynamic (ingest)
    uint64_t head;                  // packets ever enqueued
    uint64_t vbyte_end;             // virtual bytes ever enqueued
    uint32_t vcount_end;            // non-empty packets ever enqueued (mod 2^32)
    uint32_t valid_ssrc;            // FilterInvalidSSRCs state
    int64_t  last_valid_s;
    int64_t  key;                   // fKeyFrameStartPacketElementPointer as an index, -1 = NULL
    int64_t  last_nonzero;          // index of the newest non-empty packet, -1 = none
    // per tick
    int64_t  new_start;             // fFirstPacketInQueueForNewOutput, -1 = NULL
    uint64_t tail;                  // oldest index still intact in both rings
    uint64_t umin;                  // min range start over this sender's sub-streams
    uint64_t vclob;                 // bytes of the ring's virtual stream written so far (>= vbyte_end:
                                    // k_ingest's speculative copy may reach past it); slots older than
                                    // vclob - ring bytes are overwritten
    uint64_t fan_lo, fan_vlo;       // oldest packet index / vbyte the last fan-out reads
    // the last host batch (edgpu_fanout_sources): packets [batch_lo, head) came from the blob of
    // the ingest whose epoch is batch_epoch; their blob slots follow the meta ring (uint32 per
    // ring entry, same index), written by k_ingest
    uint64_t batch_lo;
    uint32_t batch_epoch, _pad_b;
    // ReflectorSocket's receive-time state (reflector_use_in_packet_receive_time, ReflectorStream.h:
    // 251-254, .cpp:1960-1994): the socket's first trailer-tagged packet of the current SSRC
    // anchors the arrival clock of every tagged packet after it
    uint32_t rt_has, rt_ssrc;       // fHasReceiveTime, fCurrentSSRC
    int64_t  rt_first_arrival;      // fFirstArrivalTime
    uint64_t rt_first_receive;      // fFirstReceiveTime
    uint32_t rt_nonmono;            // a tagged packet was enqueued: arrivals along the ring need not
                                    // be monotone, so arrival searches walk it (first_arrival_at)
    uint32_t _pad_rt;
};

// ---- Session images (cross-GPU keyframe fast start) ----
// A session image is a self-contained, position-independent copy of the part of a
// session's sender rings that a joining subscriber can still be served from: [64-B
// ImgHeader][ImgStream x ntracks][ImgSender x 2*ntracks][per sender: PktMeta x nmeta, then
// the slot bytes], every section 16-B aligned.  A delta image carries the packets after a
// given queue index instead.
constexpr uint32_t kImageMagic = 0x49474445u;   // "EDGI"
constexpr uint32_t kImageVersion = 1;
constexpr uint64_t kImageFull = ~0ull;

struct ImgHeader {                  // 64 B
    uint32_t magic, version, ntracks, nsenders;
    uint64_t bytes;                 // whole image
    int64_t  now;                   // export time (ms)
    uint32_t video_key_flag, delta;
    uint64_t _pad[3];
};

struct ImgStream {                  // 16 B
    uint64_t packet_count, _pad;
};

struct ImgSender {                  // 96 B
    uint64_t floor;                 // first queue index carried
    uint64_t head;
    uint64_t vbyte_floor;           // vbyte of `floor` (= vbyte_end when nothing is carried)
    uint64_t vbyte_end;
    uint32_t vcount_end, valid_ssrc;
    int64_t  last_valid_s;
    int64_t  key;
    int64_t  last_nonzero;
    uint64_t meta_off, bytes_off;   // from the image start
    uint32_t delta, flags;
    uint32_t nonmono;               // SenderDev.rt_nonmono: the carried arrivals need not be monotone
    uint32_t _pad;
};

struct ImgPlan {                    // one sender of one image (export or import)
    uint32_t sender;                // global sender index in this context
    uint32_t session;               // session in this context
    uint32_t ls;                    // local sender index in the session
    uint32_t first;                 // 1 for the session's first sender
    uint64_t from;                  // export: kImageFull or the first index of a delta
    uint64_t image_base;            // byte offset of the image in the buffer
    uint64_t floor, vbyte_floor, nmeta, nbytes;
    uint64_t meta_off, bytes_off;   // from the image start
    uint64_t image_bytes;           // export: size of the whole image
};

struct StreamDev {
    uint64_t packet_count;          // ReflectorStream::fPacketCount (shared by both senders)
};

struct SessionDev {
    uint32_t first_sender;          // senders of track t: first_sender + 2t (+1 for RTCP)
    uint32_t ntracks;
    uint32_t video_key_flag;        // ReflectorSession::fHasVideoKeyFrameUpdate
    uint32_t first_stream;
    // FilterInvalidSSRCs' settings, fixed when the session is set up (SetupReflectorSession's
    // inFilterSSRCs / inTimeout, QTSSReflectorModule.cpp:1457 -> ReflectorStream.cpp:1732-1767)
    uint32_t ssrc_filter;           // use_one_SSRC_per_stream
    uint32_t ssrc_timeout_s;        // timeout_stream_SSRC_secs
    // a backpressure report relocated an output (Q9) since edgpu_session_relocations last read
    // it: on a replica, the owner's next audio packet must become the audio anchor
    uint32_t relocated;
    // sticky stream errors (kStreamRingOverflow: a packet an output still needed, or the key frame
    // a new output starts at, fell out of a sender ring); the session's own outputs lose packets,
    // the tick goes on for every other session.  Read and cleared by edgpu_stream_errors.
    uint32_t errors;
};
constexpr uint32_t kStreamRingOverflow = 1u;

struct SubDev {                     // one sub-stream: subscriber x sender
    uint32_t handle;                // subscriber handle
    uint32_t sender;
    uint16_t track;
    uint8_t  kind;                  // 0 RTP, 1 RTCP
    uint8_t  transport;             // 0 UDP, 1 TCP
    uint8_t  channel;               // interleaved channel 2*track + kind (RTPStream.cpp:472-473)
    uint8_t  active;
    uint8_t  has_last;
    uint8_t  was_new;               // no bookmark when this tick began (ReflectPackets' firstPacket)
    int64_t  bookmark;              // ReflectorOutput bookmark index, -1 = none
    uint64_t last_id;               // qtssReflectorStreamLast{RTP,RTCP}PacketID
    // per tick
    uint64_t a;                     // first packet index of this tick's range
    uint64_t vstart;                // vbyte of `a`
    uint32_t vcstart;               // vcount of `a`
    uint32_t count;                 // packets to send (non-empty)
    uint64_t bytes;                 // slot bytes spanned
    uint64_t out_base;
    uint32_t desc_base;
    uint32_t nonempty;              // range [a, head) is non-empty
    // RTP-Info players (FilterPacket, RTPSessionOutput.cpp:249-280): RTP packets with
    // seq < first_seq are skipped until the client stream's first write, RTP or RTCP
    uint16_t first_seq;             // qtssRTPStrFirstSeqNumber (0 unless RTP-Info)
    uint8_t  rtp_info;              // filter armed
    uint8_t  sent_any;              // this sub-stream has written a packet (its packet count > 0)
    // egress backpressure (edgpu_fanout_blocked): the state before this tick's commit, and
    // whether the bookmarked packet is still to be sent (the next tick starts AT it)
    uint64_t prev_last_id;
    uint8_t  prev_has_last;
    uint8_t  prev_sent_any;
    uint8_t  resume_at;
    uint8_t  _pad1[5];
    // per-output rewrite (edgpu_subscriber_rewrite): kRw* flags | seq delta << 16, 0 = identity
    uint32_t rw;
    uint32_t rw_ts;                 // RTP timestamp delta (mod 2^32)
    uint32_t rw_ssrc;               // replacement SSRC (kRwSsrc), host order
    uint32_t pass;                  // the tick's copy pass that delivers this sub-stream (over-
                                    // capacity ticks; out_base / desc_base are relative to it)
};

// SubDev.rw / FanSub.rw: the per-output rewrite stage (north_star item 3).  The reference
// rewrites nothing (Q1: RTPSessionOutput::PacketShouldBeThinned returns false at
// RTPSessionOutput.cpp:685-687, the RTCP rewrite call is commented out at :600-601), so parity
// runs with rw = 0; a host that renumbers a subscriber's streams (e.g. after a source switch)
// sets it.  Every field a rewrite touches sits in a slot's first 16-B word, except an SR's RTP
// timestamp (second word).
enum : uint32_t {
    kRwActive = 1u << 0,            // any rewrite on this sub-stream
    kRwSsrc   = 1u << 1,            // replace the SSRC (RTP bytes 8-11, RTCP sender SSRC bytes 4-7)
    kRwRtcp   = 1u << 2,            // the sub-stream carries RTCP (kind 1)
};

// RTP-Info PLAY query for one track (ReflectorSession HaveStreamBuffers,
// QTSSReflectorModule.cpp:1804-1865).
struct FirstInfoQuery {
    uint32_t rtp_sender;            // the track's RTP sender
    uint32_t rtcp_sender;           // its RTCP sender for a TCP push (packets there are RTP by
                                    // port, Q12, and set HasFirstRTP too), else ~0
    int64_t  cutoff;                // now - (over-buffer - min(rtp-info offset, over-buffer))
};
struct FirstInfoResult {
    uint32_t found;                 // 0: !HasFirstRTP, 1: packet found, 2: none in the window
    uint32_t seq;                   // GetPacketRTPSeqNum of the packet
    uint32_t rtptime;               // GetPacketRTPTime (0 if len < 8)
    uint32_t _pad;
};

// One fan-out work item: up to `chunk` consecutive packets of one sender, with everything the
// copy kernel needs before it can issue the chunk's loads (k_plan_final fills it, so the
// kernel's first dependent load is this 64-B record).
struct FanWork {                    // 64 B
    uint64_t ring;                  // sender byte ring (device pointer)
    uint64_t meta;                  // sender PktMeta ring (device pointer)
    uint32_t wmask, pkmask;         // ring words - 1, ring packets - 1
    uint32_t sender;
    uint32_t np;                    // packets in the chunk
    uint32_t nw;                    // 16-B words the chunk's slots span
    uint32_t vc0;                   // vcount of the chunk's first packet
    uint32_t qb, qe;                // the sender's sub-streams: FanSub[qb, qe)
    uint64_t lo;                    // queue index of the chunk's first packet
    uint64_t vb0;                   // vbyte of the chunk's first packet
};

// Per-sub-stream copy parameters of a tick, in sender order (FanWork::qb/qe index them).
struct FanSub {                     // 48 B
    int64_t  dw;                    // arena word of virtual ring word V is dw + V
    int64_t  off;                   // wire offset of a packet with vbyte vb is off + vb
    uint64_t a;                     // first packet index this tick; ~0: nothing to send
    uint32_t ch;                    // bit 0: RTSP-interleaved; bits 8..15: channel byte
    uint32_t db;                    // descriptor index of a packet with vcount vc is db + vc
    uint32_t rw;                    // SubDev.rw
    uint32_t rw_ts;                 // timestamp delta
    uint32_t rw_ssrc_be;            // replacement SSRC as stored (big-endian bytes)
    uint32_t _pad;
};

struct TickTotals {                 // device-side, mirrors edgpu_tick_stats
    unsigned long long relayed_packets;
    unsigned long long relayed_bytes;
    unsigned long long arena_bytes;
    // the last batch's ingest counters, by ingest parity: k_ingest adds into slot seq & 1 and its
    // workgroup 0 zeroes the other slot for the next ingest (no reset launch, no "last workgroup"
    // round trip)
    unsigned long long ing_pk[2], ing_b[2];
    int status;
    unsigned int nwork;
    // cumulative (never reset)
    unsigned long long cum_relayed_packets;
    unsigned long long cum_relayed_bytes;
    unsigned long long cum_fanout_in_bytes;
    unsigned long long cum_ingested_packets;
    unsigned long long cum_ingested_bytes;
    int ingest_status;              // sticky: an ingest lapped data an in-flight fan-out reads
    unsigned int fan_next;          // dynamic fan-out variants: next work item to claim (per tick)
    unsigned int _pad;
    // measurement builds: the copy kernel's workgroups' first start / first and last exit
    // (s_memrealtime, 100 MHz) -- the tail of the dynamic schedule (EDGPU_FAN_TAIL=1 prints it)
    unsigned long long fan_t0_min, fan_done_min, fan_done_max;
    unsigned long long ing_t0_min, ing_done_min, ing_done_max;    // the same for k_ingest
    unsigned long long ing_last_span, ing_last_first;             // ... of the last finished ingest
    unsigned long long ing_ph[8], ing_last_ph[8];                 // k_ingest phase sums ([0]: segments)
    // Copy passes of an over-capacity tick (edgpu_fanout_next).  Slot k & 1 belongs to the k-th
    // launched pass: the arena bytes and descriptors its sub-streams span, and the id of the next
    // pass (kNoPass: none).  A pass's plan resets the other slot for the pass after it.
    unsigned long long pass_bytes[2];
    unsigned int pass_desc[2];
    unsigned int pass_next[2];
    unsigned int pass_slot;         // slot of the last launched pass
    unsigned int stream_errors;     // sessions newly marked with a stream error by this tick
    unsigned long long cum_lost_passes;   // passes a tick still owed when the next tick was planned
    unsigned int grow_count;        // senders this tick's plan asked to grow (GrowReq list, kMaxGrow)
    unsigned int _pad_g;
};

// A sender ring the plan found too small for the span the reference would retain (edgpu_config.
// ring_growth): the capacities it should have, as powers of two.
struct GrowReq {                    // 32 B
    uint32_t sender;
    uint32_t pk_log2;               // packets
    uint32_t bytes_log2;            // bytes
    uint32_t _pad;
    uint64_t tail, head;            // the sender's intact range when the plan measured it
};
constexpr uint32_t kMaxGrow = 1024;     // requests per tick (the rest are made again next tick)
constexpr uint32_t kNoPass = 0xFFFFFFFFu;

struct TickParams {
    int64_t  now;
    int64_t  over_buffer_ms;
    uint64_t arena_bytes;
    uint32_t max_desc;
    uint32_t nsenders;
    uint32_t nsubs;
    uint32_t nsub_blocks;
    uint32_t chunk;                 // packets per fan-out work item (per kernel variant)
    uint32_t pass_ord;              // k_plan_pass: ordinal of the pass (1, 2, ...) and its id
    uint32_t pass_id;
    uint32_t grow_on;               // ring growth: on, and its per-sender bounds
    uint32_t grow_max_pk;
    uint64_t grow_max_bytes;
    uint32_t* grow_flag;            // pinned host word (mapped): set when a request is made, so the
                                    // host learns of it without reading the tick back
};

}  // namespace edgpu
