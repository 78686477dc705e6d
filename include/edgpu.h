/*
 * edgpu.h -- C ABI of the MI355X-native batched RTP relay engine (libedgpu.so).
 *
 * The engine replaces EasyDarwin's reflector hot path behind the QTSSReflectorModule
 * plugin boundary.  Each entry point names the reference interface it stands in for
 * (paths relative to the EasyDarwin reference tree):
 *
 *   edgpu_session_add      ReflectorSession::SetupReflectorSession
 *                          (APIModules/QTSSReflectorModule/ReflectorSession.cpp:140-188) with the
 *                          SDP parse of SDPSourceInfo (APICommonCode/SDPSourceInfo.cpp:259-353)
 *   edgpu_session_remove   the end of a ReflectorSession: RemoveOutput's refcount-0 branch
 *                          (QTSSReflectorModule.cpp:2162-2192) with TearDownAllOutputs when a
 *                          broadcast stops with kill_clients (:2156-2159, ReflectorSession.cpp:
 *                          281-285)
 *   edgpu_subscriber_add   RTPSessionOutput ctor + ReflectorSession::AddOutput
 *                          (RTPSessionOutput.cpp:73-88, ReflectorSession.cpp:209-253),
 *                          i.e. QTSSReflectorModule DoSetup/DoPlay for a player
 *                          (QTSSReflectorModule.cpp:1610-1622, 1942-1946)
 *   edgpu_subscriber_play  the same for an RTP-Info player: DoPlay + HaveStreamBuffers
 *                          (QTSSReflectorModule.cpp:1804-1865, 1971-2004)
 *   edgpu_subscriber_remove ReflectorSession::RemoveOutput (ReflectorSession.cpp:255-279)
 *   edgpu_subscriber_rewrite the per-output seq / timestamp / SSRC rewrite the reference leaves
 *                          dead (RTPSessionOutput.cpp:403-561, 600-601, 685-773)
 *   edgpu_ingest           ReflectorStream::PushPacket + ReflectorSocket::ProcessPacket
 *                          (ReflectorStream.cpp:529-576, 1769-2010), called per packet by
 *                          ProcessRTPData (QTSSReflectorModule.cpp:604-678)
 *   edgpu_ingest_interleaved RTSPRequestStream::ReadRequest's '$' deframing of a pusher's
 *                          RTSP connection (Server.tproj/RTSPRequestStream.cpp:65-171) +
 *                          edgpu_ingest of the frames
 *   edgpu_keyframe_index   the keyframe index update + audio anchor inside ProcessPacket
 *                          (ReflectorStream.cpp:1876-1934, IsKeyFrameFirstPacket :1403-1513)
 *   edgpu_fanout           ReflectorSender::ReflectPackets / SendPacketsToOutput /
 *                          RTPSessionOutput::WritePacket and the egress framing of
 *                          RTPStream::Write (ReflectorStream.cpp:1024-1198,
 *                          RTPSessionOutput.cpp:564-662, Server.tproj/RTPStream.cpp:1084-1147,
 *                          RTSPSessionInterface.cpp:329-344), for every sender at once
 *   edgpu_udp_sources      the pusher RTCP-address update in ProcessPacket for UDP pushers
 *                          (ReflectorStream.cpp:1836-1866, NAT_WORKAROUND)
 *   edgpu_source_reports   ReflectorStream::SendReceiverReport on the RTCP sender's 5-s
 *                          timer (ReflectorStream.cpp:164-201, 510-527, 1039-1047)
 *
 * Conventions
 *   - Every function returns an int status using QTSS_Error values (QTSS.h:61-76):
 *     EDGPU_OK = QTSS_NoErr, EDGPU_ERR = QTSS_RequestFailed, EDGPU_BAD_ARGUMENT =
 *     QTSS_BadArgument, EDGPU_WOULD_BLOCK = QTSS_WouldBlock, plus engine-specific codes
 *     below -100 (capacity / device errors).  edgpu_last_error() gives a message.
 *   - One context per GPU.  Calls on a context are externally serialised (the reference's
 *     per-stream fBucketMutex); different contexts -- on different GPUs, or several on one GPU
 *     (replica sessions) -- may be called from different threads at the same time.
 *     edgpu_last_error() is per thread.
 *   - All device work runs on the context's HIP stream and is asynchronous unless stated.
 *     Pointers flagged EDGPU_PTR_DEVICE must stay valid until edgpu_sync() returns.
 *   - No torch or HIP types in the ABI: plain pointers and sizes.
 */
#ifndef EDGPU_H
#define EDGPU_H

#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

/* status codes (QTSS_Error-compatible where a reference counterpart exists) */
#define EDGPU_OK                 0
#define EDGPU_ERR               -1     /* QTSS_RequestFailed  */
#define EDGPU_BAD_ARGUMENT     -10     /* QTSS_BadArgument    */
#define EDGPU_WOULD_BLOCK      -14     /* QTSS_WouldBlock     */
#define EDGPU_NOT_CONNECTED    -15     /* QTSS_NotConnected   */
#define EDGPU_NO_DEVICE       -101     /* no usable gfx950 device / HIP failure */
#define EDGPU_OUT_OF_MEMORY   -102
#define EDGPU_RING_OVERFLOW   -103     /* a needed packet fell out of a sender ring */
#define EDGPU_TIMEOUT        -105     /* GPU watchdog: the device did not finish within watchdog_ms */
#define EDGPU_OUT_OVERFLOW    -104     /* a buffer too small (a fan-out sub-stream larger than the
                                          arena, a batch, a gather destination, ...) */

/* transport of a subscriber (qtssRTPTransportType, QTSS.h:219-221) */
#define EDGPU_TRANSPORT_UDP      0
#define EDGPU_TRANSPORT_TCP      1     /* RTSP-interleaved '$' framing */

/* pointer-location flags for edgpu_ingest */
#define EDGPU_PTR_HOST           0     /* host memory: copied to the device before the call returns */
#define EDGPU_PTR_DEVICE         1     /* already resident in HBM on the ctx device */
#define EDGPU_PTR_PINNED         2     /* pinned host memory from edgpu_host_alloc: copied to HBM
                                          asynchronously on the context's copy stream (below) */

/* Engine configuration.  Reflector prefs keep the reference's XML key names
 * (WinNTSupport/easydarwin.xml:131-163, read at ReflectorStream.cpp:87-117 and
 * QTSSReflectorModule.cpp:450-586); 0 selects the reference default. */
typedef struct edgpu_config {
    int32_t  device;                        /* HIP device ordinal */
    uint32_t reflector_buffer_size_sec;     /* default 1  -> 1000 ms new-client window */
    uint32_t rtp_reflector_threshold_msec;  /* default 2000, floor 1000 (relocation)   */
    uint32_t timeout_stream_SSRC_secs;      /* default 30                               */
    uint32_t use_one_SSRC_per_stream;       /* default 1 (0 = keep every SSRC) -- pass
                                               EDGPU_FALSE to disable                   */
    /* capacities (0 = default) */
    uint32_t video_ring_packets;            /* per video RTP sender, power of two (8192)  */
    uint64_t video_ring_bytes;              /* per video RTP sender, power of two (8 MiB) */
    uint32_t other_ring_packets;            /* audio/RTCP/other senders (2048)           */
    uint64_t other_ring_bytes;              /* (1 MiB)                                   */
    uint64_t out_arena_bytes;               /* fan-out output arena per tick (256 MiB)   */
    uint32_t max_out_packets;               /* descriptor capacity per tick (1 Mi)       */
    uint32_t max_batch_packets;             /* ingest batch capacity (1 Mi)              */
    uint64_t max_batch_bytes;               /* ingest blob capacity (1 GiB)              */
    uint32_t reflector_rtp_info_offset_msec; /* RTP-Info first packet: within over-buffer minus
                                               this (ReflectorStream.cpp:109-110); default 500,
                                               EDGPU_FALSE for an offset of 0 */
    /* Ring growth (default on; EDGPU_FALSE: the rings keep their configured capacities).  The
     * reference keeps every packet younger than 10 x reflector_buffer_size_sec, the key packet
     * and everything after it, and whatever a blocked output still needs, in an unbounded queue
     * (RemoveOldPackets, ReflectorStream.cpp:1233-1289, 112-114).  Each fan-out's plan measures
     * that span per sender; a sender whose span passes half of either of its rings has that ring
     * doubled (powers of two, up to the bounds below) before the next edgpu_ingest, its packets
     * moved over.  The request is noticed when the host reads the tick (edgpu_tick_stats_get /
     * edgpu_fanout_next), as every tick driver does. */
    uint32_t ring_growth;
    uint32_t max_ring_packets;              /* per sender bound of growth (1 Mi), power of two */
    uint64_t max_ring_bytes;                /* per sender bound of growth (1 GiB), power of two */
    /* reflector_use_in_packet_receive_time (default false; read once, ReflectorStream.cpp:103-104):
     * a packet longer than 12 bytes whose last 12 are "aktt" + a BE64 receive time (ms) loses
     * them, and its arrival (fTimeArrived: the new-output window, retention, relocation, transmit
     * times) becomes the socket's anchor arrival plus the receive time's offset from the anchor's
     * receive time; the anchor is the socket's first tagged packet since its SSRC -- by the
     * remote port's parity, EDGPU_PKT_REMOTE_ODD -- last changed (ReflectorSocket::ProcessPacket,
     * :1960-1994).  Arrivals further than reflector_in_packet_max_receive_sec (default 60,
     * EDGPU_FALSE for 0; :106-107, 113) ahead of the push time are clamped there. */
    uint32_t reflector_use_in_packet_receive_time;
    uint32_t reflector_in_packet_max_receive_sec;
    /* GPU watchdog (default 10000 ms; EDGPU_FALSE: unbounded): the longest any call waits for the
     * device.  A wait that runs out returns EDGPU_TIMEOUT and wedges the context: every call that
     * would enqueue work or wait returns EDGPU_TIMEOUT at once, enqueueing nothing, until the work
     * it timed out on has finished; then the context is usable again (the results of that work were
     * never read: the host re-runs or drops the tick).  edgpu_ctx_destroy waits without a bound. */
    uint32_t watchdog_ms;
    /* k_ingest's speculative copy (no reference counterpart; output bytes are the same either
     * way): a descriptor batch whose segments average at least this many packets is copied first
     * and its header words read from the copy (default 128, a 1-s C2 tick; 1: always; EDGPU_FALSE:
     * never, the header-first order).  DESIGN.md §3. */
    uint32_t ingest_spec_min;
} edgpu_config;
#define EDGPU_FALSE 0xFFFFFFFFu   /* a flag off / a value of 0 where 0 would select the default */

/* One ingested packet.  The batch blob is a sequence of 16-byte-aligned slots; a packet's
 * bytes start 4 bytes into its slot (the 4 bytes before it are the RTSP-interleaved header
 * slot the engine rewrites), so `slot` is the slot's offset / 16.  Packets of one session
 * must be contiguous and in arrival order (a pusher's TCP connection delivers exactly that);
 * `seg_offsets` (n_segments + 1 entries) splits the descriptor array into per-session
 * segments and `seg_session` names each segment's session.  A session appears in at most
 * one segment per batch. */
typedef struct edgpu_pkt_desc {
    uint32_t slot;          /* blob byte offset / 16 */
    uint16_t len;           /* packet length as received (clamped to 2060 at ingest, Q11) */
    uint8_t  channel;       /* interleaved channel: 2*track + is_rtcp */
    uint8_t  flags;         /* EDGPU_PKT_REMOTE_ODD or 0 */
    int64_t  arrival_ms;    /* OS::Milliseconds() when the packet was pushed */
} edgpu_pkt_desc;
/* A UDP push datagram from an odd source port: ProcessPacket's GetSSRC(theRemotePort & 1) reads
 * the RTCP SSRC word for it (ReflectorStream.cpp:1969; only the receive-time trailer reads it).
 * An RTSP-interleaved push has remote port 0 (PushPacket, :548, :572). */
#define EDGPU_PKT_REMOTE_ODD 1u

/* One send-ready output packet (16 bytes).  `offset` is the byte offset in the output
 * arena of the bytes to put on the wire: the UDP datagram, or the '$' ch BE16(len) frame
 * for an RTSP-interleaved subscriber. */
typedef struct edgpu_out_desc {
    uint64_t offset;
    uint32_t len;
    uint32_t packet_id;     /* low 32 bits of fStreamCountID */
} edgpu_out_desc;

/* One sub-stream (subscriber x track x RTP|RTCP) of a fan-out tick.  The table is in the
 * engine's sub-stream row order: a subscriber's rows are consecutive, in track, kind order, and
 * subscribers follow their join order, except that a subscriber may take the rows a removed
 * one left (edgpu_session_remove).  Rows of removed subscribers have desc_count 0.  Its
 * packets are desc[desc_base .. desc_base + desc_count). */
typedef struct edgpu_substream_out {
    uint32_t subscriber;    /* handle from edgpu_subscriber_add */
    uint16_t track;
    uint8_t  kind;          /* 0 RTP, 1 RTCP */
    uint8_t  transport;     /* EDGPU_TRANSPORT_* */
    uint32_t desc_base;
    uint32_t desc_count;
    uint64_t out_base;      /* arena offset of the first slot */
    uint64_t out_bytes;     /* arena bytes spanned (slot-padded) */
    uint32_t sender;        /* the engine sender (track x RTP|RTCP of a session) it relays */
    uint32_t flags;         /* EDGPU_SUB_IDENTITY: its bytes are the sender's packets unmodified
                               (UDP, no rewrite) -- two such sub-streams of one sender carry the
                               same bytes, the shorter one a suffix of the longer.
                               EDGPU_SUB_NEW: the output had no bookmark on this sender when the
                               tick began (GetBookMarkedPacket == NULL: ReflectPackets takes the
                               new-output start and sets `firstPacket`, ReflectorStream.cpp:
                               1097-1104) */
} edgpu_substream_out;
#define EDGPU_SUB_IDENTITY 1u
#define EDGPU_SUB_NEW      2u

/* Result of edgpu_fanout.  Device pointers, valid until the next edgpu_fanout.  Ticks run in
 * order on one stream: a tick's fan-out reads the rings after its own ingest and before the
 * next one (the engine had a pipelined mode that overlapped the next ingest with the fan-out;
 * it was dropped because backpressure reports and arrivals of the overlapped batch arrived a
 * tick late -- the pushers' H2D copies still overlap through edgpu_ingest_host). */
typedef struct edgpu_fanout_result {
    const uint8_t*              arena;          /* device */
    const edgpu_out_desc*       desc;           /* device */
    const edgpu_substream_out*  substreams;     /* device */
    uint32_t                    n_substreams;
} edgpu_fanout_result;

/* Per-tick totals, read back by edgpu_tick_stats_get (which syncs). */
typedef struct edgpu_tick_stats {
    uint64_t relayed_packets;   /* IncrementTotalPackets semantics (RTPStream.cpp:1213-1216) */
    uint64_t relayed_bytes;     /* wire bytes incl. '$' framing (of the passes copied so far) */
    uint64_t arena_bytes;       /* slot bytes of the whole tick (every pass) */
    uint64_t ingested_packets;  /* the batch the last edgpu_keyframe_index indexed (the counters
                                   move at the index, not at edgpu_ingest) */
    uint64_t ingested_bytes;
    int32_t  status;            /* device-side error of the whole tick (EDGPU_OUT_OVERFLOW, ...); a
                                   ring that lost a packet one session needed marks that session
                                   instead (stream_errors) */
    uint32_t _pad;
    /* the current copy pass (edgpu_fanout_next): arena bytes and descriptors the result's
     * sub-streams span, its ordinal (0 = the pass edgpu_fanout launched) and whether another
     * pass follows */
    uint64_t pass_arena_bytes;
    uint32_t pass_packets;
    uint32_t pass;
    uint32_t more_passes;
    /* sessions the tick newly marked with a stream error (edgpu_stream_errors): their outputs
     * lost packets, every other session's went out as usual */
    uint32_t stream_errors;
} edgpu_tick_stats;

typedef struct edgpu_ctx edgpu_ctx;

const char* edgpu_version(void);
const char* edgpu_last_error(void);
void        edgpu_config_default(edgpu_config* cfg);

int  edgpu_ctx_create(const edgpu_config* cfg, edgpu_ctx** out);
int  edgpu_ctx_destroy(edgpu_ctx* ctx);
int  edgpu_sync(edgpu_ctx* ctx);

/* Push sessions.  `udp_push` = 0 for an RTSP-interleaved (TCP) push, 1 for UDP push
 * (then the RTCP socket is bound on an odd port and only SRs are accepted, Q12/Q14). */
int  edgpu_session_add(edgpu_ctx* ctx, const char* sdp, uint32_t sdp_len, int udp_push,
                       uint32_t* out_session);
int  edgpu_session_tracks(edgpu_ctx* ctx, uint32_t session, uint32_t* out_tracks);
/* The session's SSRC filter settings: SetupReflectorSession takes use_one_SSRC_per_stream and
 * timeout_stream_SSRC_secs per session, from the module prefs as they are when the session is set
 * up (QTSSReflectorModule.cpp:1457, RereadPrefs :478-481 -> FilterInvalidSSRCs,
 * ReflectorStream.cpp:1732-1767).  edgpu_session_add gives a session the context's
 * edgpu_config values; this changes them (before its first packet, for a session a module set up
 * after a RereadPrefs).  Both are taken as given (a timeout of 0 s is the reference's too). */
int  edgpu_session_ssrc_prefs(edgpu_ctx* ctx, uint32_t session, uint32_t use_one_SSRC_per_stream,
                              uint32_t timeout_stream_SSRC_secs);

/* Destroys a push session -- what the reference does when a ReflectorSession's reference
 * count reaches 0 (its pusher gone, every output removed: RemoveOutput, QTSSReflectorModule.cpp:
 * 2133-2196).  The reference counting itself is the host's (the module's session map): the
 * engine keeps a session, its queues, packet ids, key pointers and SSRC latch, for as long as
 * the host does -- a pusher that reconnects to a session its players kept alive continues it
 * (FindOrCreateSession, :1479-1536), a pusher after edgpu_session_remove gets a fresh one from
 * edgpu_session_add (ids from 1, unlatched SSRC filter, empty queues).
 * flags: EDGPU_SESSION_KILL_OUTPUTS removes the session's subscribers with it
 * (kill_clients_when_broadcast_stops: TearDownAllOutputs, :2156-2159; their handles become
 * invalid); without it the call fails with EDGPU_ERR while a subscriber is attached.
 * Frees the session's HBM rings.  The session id, and its sender / stream table rows, are
 * reused by a later edgpu_session_add of a session with as many tracks; a removed subscriber's
 * sub-stream rows are reused by a later subscriber of a session with as many tracks
 * (subscriber handles are never reused).  Fails while an ingest is pending a keyframe index.
 * Syncs (a fan-out copy in flight may still read the rings). */
#define EDGPU_SESSION_KILL_OUTPUTS 1u
int  edgpu_session_remove(edgpu_ctx* ctx, uint32_t session, uint32_t flags);

/* The SDP parse edgpu_session_add applies (host only, no context, no GPU): the restatement of
 * SDPSourceInfo::Parse (APICommonCode/SDPSourceInfo.cpp:172-420) -- one track per line
 * starting with 'm', its payload type (1 video, 2 audio, 0 other), its rtpmap payload name
 * (the text the H.264 keyframe gate compares, ReflectorStream.cpp:1879, Q3) and its trackID
 * (a=control, else its position).  Names longer than 244 bytes are truncated here (not in the
 * session).  *n_tracks receives the count; EDGPU_BAD_ARGUMENT if it exceeds `cap`. */
typedef struct edgpu_sdp_track {
    uint32_t payload_type;
    uint32_t track_id;
    uint32_t name_len;
    char     name[244];
} edgpu_sdp_track;
int  edgpu_sdp_parse(const char* sdp, uint32_t sdp_len, edgpu_sdp_track* out, uint32_t cap, uint32_t* n_tracks);

/* Subscribers: a join takes effect at the next edgpu_fanout, like a new output being
 * picked up by the next ReflectPackets. */
int  edgpu_subscriber_add(edgpu_ctx* ctx, uint32_t session, int transport,
                          uint32_t* out_handle);
int  edgpu_subscriber_remove(edgpu_ctx* ctx, uint32_t handle);
/* The subscriber's place in its session's bucket arrays, as ReflectorStream::AddOutput /
 * FindBucket give it (ReflectorStream.cpp:281-334: the first empty place, 16 per bucket, a
 * removed output's place reused): its writes' transmit times are bucket x
 * reflector_bucket_offset_delay_msec early (ReflectorStream.cpp:1107, RTPSessionOutput.cpp:
 * 603-608), and a new output's first write decides for every output after it in this order
 * (ReflectorStream.cpp:1088-1104).  Used by the egress's write gate (edgpu_egress_pacing). */
int  edgpu_subscriber_slot(edgpu_ctx* ctx, uint32_t handle, int32_t* out_slot);
/* A burst of joins (e.g. BASELINE config C4's 10k mid-GOP joins) in one call: subscriber i
 * joins sessions[i] with transports[i]; handles as edgpu_subscriber_add would return them. */
int  edgpu_subscribers_add(edgpu_ctx* ctx, uint32_t n, const uint32_t* sessions,
                           const int32_t* transports, uint32_t* out_handles);

/* PLAY of a player that needs RTP-Info (DoPlay's rtpInfoEnabled branch,
 * QTSSReflectorModule.cpp:1867-2023: the kRequiresRTPInfoSeqAndTime player profile, user
 * agents "Android" and "vlc").  For every track, HaveStreamBuffers (:1804-1865) needs a
 * received RTP packet (HasFirstRTP) and a first packet no older than reflector_buffer_size
 * minus reflector_rtp_info_offset_msec at `now_ms` (ReflectorSender::GetFirstPacketInfo,
 * ReflectorStream.cpp:728-753).  Its sequence number and RTP timestamp go to out_info[track]
 * (the PLAY response's RTP-Info), and until the player's first write on a track, RTP packets
 * with a lower sequence number are not sent to it (FilterPacket, RTPSessionOutput.cpp:249-280;
 * a plain 16-bit compare).  If a track has nothing buffered, no subscriber is added and
 * EDGPU_WOULD_BLOCK is returned: the reference retries the PLAY from a 100 ms idle timer
 * (:1985-2003).  Ingested packets must be indexed (edgpu_keyframe_index) first.
 * flags: 0 (then this is edgpu_subscriber_add) or EDGPU_PLAY_RTP_INFO. */
#define EDGPU_PLAY_RTP_INFO 1u
typedef struct edgpu_rtp_info {
    uint16_t seq;           /* qtssRTPStrFirstSeqNumber */
    uint16_t _pad;
    uint32_t rtptime;       /* qtssRTPStrFirstTimestamp */
} edgpu_rtp_info;
int  edgpu_subscriber_play(edgpu_ctx* ctx, uint32_t session, int transport, uint32_t flags,
                           int64_t now_ms, uint32_t* out_handle, edgpu_rtp_info* out_info);

/* Per-output rewrite stage (north_star item 3).  From the next edgpu_fanout, every packet
 * written to subscriber `handle`'s track `track` is rewritten in flight:
 *   RTP sub-stream:  sequence number += seq_delta (mod 2^16), timestamp += ts_delta (mod 2^32),
 *                    SSRC = ssrc when flags has EDGPU_REWRITE_SSRC -- for packets of >= 12 bytes;
 *   RTCP sub-stream: sender SSRC (bytes 4-7) = ssrc with EDGPU_REWRITE_SSRC (>= 8 bytes), and the
 *                    RTP timestamp of a sender report (PT 200, bytes 16-19) += ts_delta (>= 20 B).
 * CSRC lists, extensions and payloads are never touched; lengths and descriptors are unchanged.
 * NULL (or all-zero deltas without EDGPU_REWRITE_SSRC) is the identity, the default.  The
 * reference never rewrites (Q1: RTPSessionOutput::PacketShouldBeThinned returns false at
 * RTPSessionOutput.cpp:685-687, and the RTCP rewrite RewriteRTCP / TrackRTCPPackets,
 * :403-561, is not called, :600-601), so parity runs use the identity; FilterPacket's first-seq
 * test and an RTP-Info PLAY's reply see the source's sequence numbers (a host that rewrites an
 * RTP-Info player's stream adjusts its RTP-Info header by the same deltas). */
#define EDGPU_REWRITE_SSRC 1u
typedef struct edgpu_rewrite {
    uint16_t seq_delta;
    uint16_t flags;
    uint32_t ts_delta;
    uint32_t ssrc;          /* host order */
} edgpu_rewrite;
int  edgpu_subscriber_rewrite(edgpu_ctx* ctx, uint32_t handle, uint32_t track, const edgpu_rewrite* rw);

int  edgpu_ingest(edgpu_ctx* ctx, const edgpu_pkt_desc* desc, uint32_t n_packets,
                  const uint32_t* seg_offsets, const uint32_t* seg_session,
                  uint32_t n_segments, const uint8_t* blob, uint64_t blob_bytes,
                  int ptr_location);

/* Pinned host staging for edgpu_ingest (north_star: "C++ host code batches ingested RTP
 * packets ... into pinned HBM ring buffers"; replaces the per-packet memcpy into a
 * ReflectorPacket, ReflectorStream.h:104-114).  The host (its socket reader) writes a batch --
 * descriptors, segments and the slot blob -- straight into buffers from edgpu_host_alloc and
 * calls edgpu_ingest(..., EDGPU_PTR_PINNED): the batch is validated on the host, copied to one
 * of two device staging sets on a dedicated copy stream, and k_ingest waits for that copy on
 * the context stream -- so the PCIe transfer of batch t+1 overlaps the fan-out of batch t, and
 * the call returns without waiting for the GPU.  Buffer reuse: a pinned batch may be rewritten
 * once the NEXT ingest call (edgpu_ingest of any pointer kind, or edgpu_ingest_interleaved), or
 * any call that synchronises the context (edgpu_sync, edgpu_tick_stats_get), has returned --
 * every ingest entry point waits for the previous pinned batch's copy, and the context stream
 * waits for it before its ingest kernel -- so two host batches used alternately never stall the
 * reader on the GPU.  edgpu_host_alloc / edgpu_host_free
 * may be called from any thread (a pusher growing its blob); a free waits for the copy stream. */
int  edgpu_host_alloc(edgpu_ctx* ctx, uint64_t bytes, void** out);
int  edgpu_host_free(edgpu_ctx* ctx, void* ptr);
/* Copies bytes [offset, offset + bytes) of the NEXT pinned batch's blob to the device ahead of
 * its edgpu_ingest(..., EDGPU_PTR_PINNED), on the copy stream, while the host is still filling
 * the rest: a host whose pushers write the blob in slabs streams each finished prefix (the
 * QTSS module drop-in does, reflector_adapter.cpp), and the ingest call then copies only the
 * remainder.  Ranges must extend the prefix staged so far (offset == bytes already staged) and
 * those bytes must not change before the ingest (a blob moved to a larger buffer keeps them).
 * May be called from another thread than the context's other calls.  A pinned batch that
 * edgpu_ingest refuses for its size or structure drops what was copied ahead of it; offset 0 with
 * bytes 0 drops it explicitly (a host whose batch came to nothing, e.g. every packet of it belonged
 * to a session removed since: the next pinned batch is then copied whole). */
int  edgpu_ingest_prestage(edgpu_ctx* ctx, const uint8_t* blob, uint64_t offset, uint64_t bytes);
/* RTSP-interleaved push ingest: the pusher connections' raw TCP reads, deframed on the GPU.
 * Replaces RTSPRequestStream::ReadRequest's '$' branch (Server.tproj/RTSPRequestStream.cpp:
 * 65-171, RTSPSession.cpp:240-262) and the per-frame hand-off to ProcessRTPData
 * (RTSPSession.cpp:2131-2178, QTSSReflectorModule.cpp:604-678): each connection's bytes are
 * split into '$' ch BE16(len) frames, frame i of a session becomes a packet on channel `ch`
 * (track ch/2, RTCP when odd) with the arrival time of the read that completed it, and the
 * packets are ingested exactly as edgpu_ingest would (same batch semantics; run
 * edgpu_keyframe_index next).  A frame split across calls is carried on the device (at most
 * 2046 bytes per session).
 *
 * reads[i] is one read of session reads[i].session (an RTSP-interleaved, udp_push = 0
 * session): `len` bytes at bytes + offset.  A session's reads are consecutive entries of
 * `reads`, in arrival order, and contiguous in `bytes`.  `bytes` is host memory
 * (EDGPU_PTR_HOST, staged) or device memory on the ctx GPU (EDGPU_PTR_DEVICE, 16-B aligned).
 *
 * results[i] (host memory) reports read i: `frames` it completed, `consumed` bytes the engine
 * took (framed or carried), and `status`:
 *   EDGPU_TCP_MESSAGE  a non-'$' byte at a frame boundary: an RTSP request (e.g. a
 *                      SET_PARAMETER keep-alive or TEARDOWN) starts at byte `consumed` of this
 *                      read; the rest of this read and the session's later reads in this call
 *                      are the host RTSP stack's.  The session's carry is cleared.
 *   EDGPU_TCP_DROPPED  a frame longer than the 2047-byte request buffer: the reference asks the
 *                      socket for 0 bytes and treats the connection as closed (Socket.cpp:
 *                      383-388); set on the read that fills the buffer and later reads.
 * `carry` is the session's carried byte count after the call.  Returns EDGPU_OUT_OVERFLOW
 * (nothing ingested, no carry changed) when the frames exceed max_batch_packets.  Host reads
 * are staged in a max_batch_bytes buffer; device reads are read in place (the frames are
 * copied from them into the sender rings).  Returns once the frames are found and `results`
 * written, which is before the copy into the rings has run (it is stream-ordered before the
 * context's next work): device `bytes`, like every EDGPU_PTR_DEVICE pointer, stay valid until
 * edgpu_sync (or a synchronising call) returns; host `bytes` are consumed on return. */
#define EDGPU_TCP_MESSAGE  1
#define EDGPU_TCP_DROPPED  2
typedef struct edgpu_tcp_read {
    uint32_t session;
    uint32_t len;
    uint64_t offset;        /* byte offset of the read in `bytes` */
    int64_t  arrival_ms;    /* OS::Milliseconds() when the read returned */
} edgpu_tcp_read;
typedef struct edgpu_tcp_result {
    uint32_t frames;
    uint32_t consumed;
    int32_t  status;        /* 0, EDGPU_TCP_MESSAGE or EDGPU_TCP_DROPPED */
    uint32_t carry;
} edgpu_tcp_result;
int  edgpu_ingest_interleaved(edgpu_ctx* ctx, const edgpu_tcp_read* reads, uint32_t n_reads,
                              const uint8_t* bytes, uint64_t n_bytes, int ptr_location,
                              edgpu_tcp_result* results);

/* Closes the ingested batch (the keyframe index itself runs inside the ingest kernel, after each
 * segment's packets are enqueued); required between an ingest and the next call. */
int  edgpu_keyframe_index(edgpu_ctx* ctx);
int  edgpu_fanout(edgpu_ctx* ctx, int64_t now_ms, edgpu_fanout_result* out);

/* Over-capacity ticks.  A tick whose outputs exceed out_arena_bytes or max_out_packets is not
 * dropped: it is delivered in copy passes over consecutive rows of the sub-stream table, each
 * within the arena and the descriptor array (the reference walks every output of every sender in
 * each ReflectPackets, ReflectorStream.cpp:1088-1120, so no output may lose a tick).  edgpu_fanout
 * launches pass 0; the result then shows only that pass's sub-streams (the other rows have
 * desc_count 0 and out_bytes 0; flags are set on every row), their out_base / desc_base relative to
 * the pass's arena and descriptors.  After consuming a pass the host calls edgpu_fanout_next:
 * *launched = 1 when it launched the next pass (`out` as above), 0 when the tick is complete.
 * edgpu_tick_stats_get reports the current pass (pass_arena_bytes, pass_packets, more_passes).
 * Every pass of a tick must be consumed before the next edgpu_fanout and edgpu_session_remove:
 * those fail with EDGPU_ERR while a pass is owed (session removal reads that from the device when
 * the host has not read the tick's stats; edgpu_counters.lost_passes counts passes a tick still
 * owed when the next tick was planned).  edgpu_ingest / edgpu_ingest_interleaved fail the same
 * way while the host knows of an owed pass; before it has read the stats an ingest may run, and a batch that would lap the tick's window in a ring while a pass is
 * owed fails the ring (EDGPU_RING_OVERFLOW) instead of corrupting the pass.  Subscribers may come and go between passes: the passes keep the tick's table (rows
 * added since are not in it, rows of removed subscribers still deliver the tick, and their rows
 * are reused only from the next tick).  Backpressure reports (edgpu_fanout_blocked) take
 * tick-wide sub-stream rows and may follow any pass.  A tick fits one pass whenever its bytes and descriptors do; a single
 * sub-stream larger than the arena (out_arena_bytes below a sender ring) still fails the tick
 * with EDGPU_OUT_OVERFLOW. */
int  edgpu_fanout_next(edgpu_ctx* ctx, edgpu_fanout_result* out, uint32_t* launched);

/* Egress backpressure.  The host writes a tick's sub-streams to their sockets; when a socket
 * stops accepting (EAGAIN -> QTSS_WouldBlock, RTPStream::Write -> RTPSessionOutput::
 * WritePacket, RTPSessionOutput.cpp:600-615) after `sent` of the sub-stream's desc_count
 * packets, report it here, after edgpu_fanout and before the next edgpu_ingest.  The engine
 * then keeps the state ReflectorSender::SendPacketsToOutput leaves for a blocked output
 * (ReflectorStream.cpp:1138-1198): the bookmark is the blocked packet -- moved to the key
 * frame when it is older than rtp_reflector_threshold_msec and the key frame is newer
 * (NeedRelocateBookMark, :1293-1322, Q9; the session's video-key flag is set, so the next
 * audio packet becomes the audio anchor) -- the last-sent packet id is the last packet
 * written, and the next edgpu_fanout resumes at the bookmark.  The tick's relayed counters
 * drop the unsent packets.  `substream` indexes the tick's edgpu_substream_out table.
 * Reports with sent >= desc_count are no-ops. */
typedef struct edgpu_blocked {
    uint32_t substream;
    uint32_t sent;
} edgpu_blocked;
int  edgpu_fanout_blocked(edgpu_ctx* ctx, const edgpu_blocked* reports, uint32_t n);

/* ---- UDP pushers: source addresses and receiver reports ----
 * A UDP push session (edgpu_session_add udp_push=1) receives datagrams on a bound even/odd
 * port pair; the host's socket reader passes the packets to edgpu_ingest (channel =
 * 2*track + 1 for the odd, RTCP port) and, in the same arrival order, their source
 * addresses here -- ReflectorSocket::ProcessPacket's remote address (ReflectorStream.cpp:
 * 1769-1866).  The engine keeps each track's pusher RTCP address as the reference does
 * with NAT_WORKAROUND (ReflectorStream.h:63, .cpp:1843-1855): set by the first datagram,
 * moved by every RTCP-port datagram that passes the SR-only gate (RTCPPacket::ParsePacket
 * + type 200, Q14), an even RTP source port followed by +1.  Datagrams from address 0,
 * empty ones and tracks out of range change nothing.  `head` = the datagram's first 4
 * bytes (what the SR gate reads with `len`).  Only RTCP datagrams and a track's first RTP
 * datagram can change the address, so a reader may pass just those.
 * Replaces: the fDestRTCPAddr/fDestRTCPPort update inside ReflectorSocket::ProcessPacket. */
typedef struct edgpu_udp_source {
    uint32_t session;
    uint8_t  channel;
    uint8_t  _pad;
    uint16_t port;        /* host order */
    uint32_t addr;        /* IPv4, host order */
    uint32_t len;
    uint8_t  head[4];
} edgpu_udp_source;
int  edgpu_udp_sources(edgpu_ctx* ctx, const edgpu_udp_source* src, uint32_t n);

/* Receiver reports to UDP pushers.  Every edgpu_fanout(now) runs, for each track, the RTCP
 * sender's report timer (ReflectorSender::ReflectPackets, ReflectorStream.cpp:1039-1047):
 * when now > last + kRRInterval (5000 ms) the timer restarts at now and, if the pusher's
 * RTCP address is known, one report is queued -- ReflectorStream::SendReceiverReport
 * (:510-527): RR (header + SSRC), SDES CNAME, and the 'QTSS' APP packet carrying the eye
 * count (client subscribers of the session, ReflectorSession.cpp:215-268) twice, built as
 * the ReflectorStream constructor lays it out (:164-201).  edgpu_source_reports returns the
 * reports queued by the last edgpu_fanout (session then track order) for the host to send
 * from the track's RTCP socket to (addr, port).
 * Identity: the reference draws the report SSRC from rand() and the CNAME from
 * OS::Milliseconds()/1000 when the stream is created (RTCPSRPacket.cpp:87-117); the engine
 * does the same at edgpu_session_add, and edgpu_source_identity overrides both. */
#define EDGPU_RR_MAX 96
typedef struct edgpu_source_report {
    uint32_t session;
    uint16_t track;
    uint16_t port;        /* host order */
    uint32_t addr;        /* IPv4, host order */
    uint32_t len;
    uint8_t  bytes[EDGPU_RR_MAX];
} edgpu_source_report;
int  edgpu_source_reports(edgpu_ctx* ctx, edgpu_source_report* out, uint32_t cap, uint32_t* n_out);
int  edgpu_source_identity(edgpu_ctx* ctx, uint32_t session, uint32_t track, uint32_t ssrc,
                           int64_t cname_secs);
/* Subscribers of `session` served by other contexts (replica sessions on other GPUs, §8.e):
 * the owner's eye count is its own clients plus these, as the single reference process
 * counts every output (IncEyeCount / DecEyeCount).  `delta` is +1 per remote join, -1 per
 * remote leave. */
int  edgpu_session_eyes_add(edgpu_ctx* ctx, uint32_t session, int32_t delta);
/* The same for a remote subscriber that also takes its place in the owner's bucket arrays
 * (ReflectorStream::AddOutput / RemoveOutput, ReflectorStream.cpp:281-336: the first empty place,
 * 16 a bucket), so that the owner's and its replicas' subscribers of one session are numbered
 * in one array, as the reference numbers them in one process: a subscriber past the first
 * bucket then gets the reference's bucket lateness in its transmit times on whichever GPU serves
 * it.  edgpu_session_remote_join counts the eye and returns the place; the replica passes it to
 * edgpu_subscriber_set_slot for its subscriber.  edgpu_session_remote_leave frees it. */
int  edgpu_session_remote_join(edgpu_ctx* ctx, uint32_t session, int32_t* out_place);
int  edgpu_session_remote_leave(edgpu_ctx* ctx, uint32_t session, int32_t place);
/* Moves a subscriber to bucket place `slot` of its session (a replica session's subscriber takes
 * the place its owner gave it, edgpu_session_remote_join).  Fails if another output holds it. */
int  edgpu_subscriber_set_slot(edgpu_ctx* ctx, uint32_t handle, int32_t slot);

/* ---- Socket egress (host side) ----
 * Sends a fan-out tick to the subscribers' sockets as RTPStream::Write does
 * (Server.tproj/RTPStream.cpp:1084-1147): UDP datagrams through the sub-stream's RTP / RTCP
 * socket with send errors ignored (a full socket drops the datagram, as the reference's
 * (void)SendTo); RTSP-interleaved frames on the subscriber's RTSP connection with
 * RTSPResponseStream::WriteV(kAllOrNothing) semantics (RTSPResponseStream.cpp:36-140: a frame
 * that goes out in part counts as sent and its tail is buffered; a frame that gets no byte
 * blocks).  Blocked TCP sub-streams are reported with edgpu_fanout_blocked before returning.
 * The tick's distinct bytes come over PCIe in one copy (identity UDP sub-streams of a sender share
 * one region, edgpu_arena_gather), with the descriptors and sub-stream table; `threads` workers
 * own disjoint subscribers and send with sendmmsg / sendmsg.  An over-capacity tick is sent pass
 * by pass (the call runs edgpu_fanout_next itself), so `r` is the result of edgpu_fanout.
 *
 * UDP loss granularity.  By default (EDGPU_EGRESS_GSO unset or 1) runs of equal-length
 * datagrams of a sub-stream (FU-A fragments of a frame) leave as UDP GSO messages (UDP_SEGMENT,
 * up to 64 datagrams / 64 KiB each): the wire carries exactly the datagrams the reference
 * sends, but a send the socket refuses (EAGAIN / ENOBUFS) drops the whole message, where the
 * reference's per-packet (void)SendTo drops one datagram (RTPStream.cpp:1145).  What arrives is
 * always an in-order subset of the tick's datagrams per sub-stream (no reordering, no
 * duplicates; tests/test_gpu_egress.py).  EDGPU_EGRESS_GSO=0 is the reference-exact mode: one
 * datagram per message, one datagram lost per refused send. */
typedef struct edgpu_egress edgpu_egress;
typedef struct edgpu_egress_stats {
    uint64_t udp_datagrams, udp_bytes;
    uint64_t udp_dropped;       /* SendTo failures, ignored like the reference */
    uint64_t tcp_frames, tcp_bytes;
    uint32_t blocked_substreams;
    uint32_t _pad;
    double   copy_ms, send_ms;  /* device -> pinned host copy; socket writes */
    uint64_t copied_bytes;      /* bytes brought over PCIe for this tick */
    uint64_t stale_dropped;     /* paced subscribers: stale TCP non-video RTP packets dropped (Q20) */
} edgpu_egress_stats;
int  edgpu_egress_create(edgpu_ctx* ctx, uint32_t threads, edgpu_egress** out);
int  edgpu_egress_destroy(edgpu_egress* eg);
const char* edgpu_egress_last_error(edgpu_egress* eg);
/* UDP subscriber track: datagrams leave through rtp_fd / rtcp_fd (-1: a per-worker socket) to
 * ipv4:port (network byte order, as in sockaddr_in). */
int  edgpu_egress_udp(edgpu_egress* eg, uint32_t subscriber, uint32_t track, int rtp_fd, int rtcp_fd,
                      uint32_t ipv4_be, uint16_t rtp_port_be, uint16_t rtcp_port_be);
/* RTSP-interleaved subscriber: its (non-blocking) RTSP connection. */
int  edgpu_egress_tcp(edgpu_egress* eg, uint32_t subscriber, int fd);
int  edgpu_egress_send(edgpu_egress* eg, const edgpu_fanout_result* r, edgpu_egress_stats* out);
/* The (sub-stream, sent) backpressure reports of the last edgpu_egress_send (*n = count). */
int  edgpu_egress_blocked(edgpu_egress* eg, edgpu_blocked* out, uint32_t cap, uint32_t* n);
/* Writes buffered TCP tails that fit now; *pending = bytes still buffered. */
int  edgpu_egress_flush(edgpu_egress* eg, uint64_t* pending);
/* Subscribers whose RTSP connection failed with an error other than EAGAIN since the last
 * call (reset / closed peer): their frames are no longer written (the reference counts such a
 * write as done, RTPSessionOutput.cpp:612-653); the host tears the session down
 * (ClientSessionClosing -> edgpu_subscriber_remove).  Sockets are written with MSG_NOSIGNAL. */
int  edgpu_egress_disconnected(edgpu_egress* eg, uint32_t* out, uint32_t cap, uint32_t* n);

/* ---- The server's write gate (Q20): over-buffer window and TCP-audio thinning ----
 * Behind the reference module, each relayed packet goes through the server's RTPStream::Write
 * (Server.tproj/RTPStream.cpp:1048-1147) with the transmit time RTPSessionOutput::WritePacket gave
 * it (RTPSessionOutput.cpp:603-608: now - bucket lateness, + the output's buffer delay left for the
 * packet).  There the session's over-buffer window (RTPOverbufferWindow::CheckTransmitTime) holds a
 * packet whose time has not come -- QTSS_WouldBlock: the output stops for this reflect, and on a new
 * output's first pass the packet's age becomes its buffer delay (RTPSessionOutput.cpp:612-622) --
 * and RTPStream::UpdateQualityLevel (:936-1045) drops RTP packets of a TCP non-video stream that have
 * fallen more than drop_all_packets_delay behind.  With pacing on for a subscriber the egress does
 * the same before its socket writes: held packets are reported to the engine like a blocked socket
 * (edgpu_fanout_blocked), dropped ones count as written.  It needs each packet's arrival (so serial
 * ticks: edgpu_fanout_arrivals) and the tick's clock (edgpu_egress_clock), the subscriber's bucket
 * place comes from the engine (edgpu_subscriber_slot). */
#define EDGPU_PACE_OVERBUFFER 1u   /* the client asked for dynamic rate (x-dynamic-rate: 1): the
                                      reflector otherwise turns overbuffering off, QRM:1772-1777 */
typedef struct edgpu_pacing {
    int64_t  play_time_ms;         /* the PLAY's time (RTPSession::fPlayTime): packets due before it
                                      are never thinned (RTPStream.cpp:941-942) */
    uint32_t video_tracks;         /* bit t: track t is video (never thinned, :946-948) */
    uint32_t flags;                /* EDGPU_PACE_* */
} edgpu_pacing;
/* Server and reflector prefs the gate reads; edgpu_egress_create sets the reference defaults
 * (QTSServerPrefs.cpp: send_interval 50, max_send_ahead_time 25, overbuffer_rate 2.0,
 * drop_all_packets_delay 2500, thin_all_the_way_delay 1500, start_thinning_delay 0; the late
 * tolerance's 1.5-s default adjusts none, RTPStream.cpp:897-918; the reflector's bucket offset
 * delay 73 ms, 16 outputs a bucket, buffer 1000 ms, ReflectorStream.cpp:53-117). */
typedef struct edgpu_pacing_config {
    int64_t  bucket_delay_ms;      /* reflector_bucket_offset_delay_msec */
    int64_t  over_buffer_ms;       /* reflector_buffer_size_sec x 1000: a new output's buffer delay */
    int64_t  drop_all_packets_ms, thin_all_the_way_ms, start_thinning_ms;
    uint32_t bucket_size;          /* outputs per bucket (16) */
    uint32_t send_interval_ms, max_send_ahead_s;
    float    overbuffer_rate;
} edgpu_pacing_config;
/* (A subscriber's over-buffer window takes send_interval_ms, max_send_ahead_s, overbuffer_rate and
 * over_buffer_ms when edgpu_egress_pacing turns its gate on, as an RTPSession builds its window at
 * SETUP; the other fields apply at every send.) */
int  edgpu_egress_pacing_config(edgpu_egress* eg, const edgpu_pacing_config* cfg);
/* Turns the gate on for `subscriber` (NULL: off).  Call after its edgpu_egress_udp / _tcp. */
int  edgpu_egress_pacing(edgpu_egress* eg, uint32_t subscriber, const edgpu_pacing* p);
/* The tick's clock (OS::Milliseconds at the reflect), for the next edgpu_egress_send. */
int  edgpu_egress_clock(edgpu_egress* eg, int64_t now_ms);
/* Why each sub-stream of the last edgpu_egress_send stopped: `sent` descriptors went (written,
 * or dropped as stale), `written` of them reached the socket; cause 0 = the socket would block,
 * 1 = the write gate held the next packet. */
typedef struct edgpu_egress_block {
    uint32_t substream, sent, written, cause;
} edgpu_egress_block;
int  edgpu_egress_block_info(edgpu_egress* eg, edgpu_egress_block* out, uint32_t cap, uint32_t* n);

/* Per-stream error isolation (a bad stream marks that stream, not the batch).  A
 * sender ring too small for what a session's outputs still need -- a blocked output's bookmark
 * or a new output's key frame overwritten by newer packets (the reference's queue is unbounded,
 * ReflectorStream.cpp:1088-1120) -- marks the session; its outputs resume at the oldest packet
 * still held (a new output waits for the next tick), and every other session's tick is
 * unaffected.  Lists the marked live sessions (code EDGPU_RING_OVERFLOW) and clears the marks of
 * those returned; *n = how many are marked.  Syncs. */
int  edgpu_stream_errors(edgpu_ctx* ctx, uint32_t* sessions, int32_t* codes, uint32_t cap, uint32_t* n);

int  edgpu_tick_stats_get(edgpu_ctx* ctx, edgpu_tick_stats* out);   /* syncs; EDGPU_ERR while an
                                                                       ingest awaits its index */

/* The arrival time (fTimeArrived, OS::Milliseconds() at PushPacket) of each descriptor of
 * the current copy pass of the last edgpu_fanout: out[i] for desc[i], i < the pass's
 * pass_packets (serial ticks; call before the next edgpu_fanout / edgpu_fanout_next).
 * RTPSessionOutput::WritePacket derives the
 * QTSS_PacketStruct transmit time from it (RTPSessionOutput.cpp:604-608), which the server's
 * RTPStream::Write hands to its thinning and over-buffer logic (RTPStream.cpp:1062,1119-1137).
 * `out` is host memory (ptr_kind EDGPU_PTR_HOST) or device memory (EDGPU_PTR_DEVICE); `n`
 * must be at least the pass's descriptors. */
int  edgpu_fanout_arrivals(edgpu_ctx* ctx, int64_t* out, uint32_t n, int ptr_kind);
/* edgpu_fanout_arrivals and / or, per descriptor of the current pass, the blob slot (byte offset /
 * 16) of its packet in the batch of the LAST edgpu_ingest -- when that was a host batch
 * (EDGPU_PTR_PINNED or EDGPU_PTR_HOST) and the packet came with it -- else EDGPU_NO_SOURCE.  A host
 * that still holds that blob can read an identity UDP descriptor's bytes (the packet, `len` bytes)
 * at blob + slot * 16 + 4 instead of reading the arena back (the module adapter does); for other
 * sub-streams the arena's bytes differ (framing, rewrite).  Either output may be NULL; serial
 * ticks; syncs. */
#define EDGPU_NO_SOURCE 0xFFFFFFFFu
int  edgpu_fanout_packet_info(edgpu_ctx* ctx, int64_t* arrivals, uint32_t* sources, uint32_t n, int ptr_kind);

/* What a host write loop needs of one descriptor, in one row: the descriptor, its packet's
 * arrival (edgpu_fanout_arrivals) and batch slot (edgpu_fanout_packet_info's sources). */
typedef struct edgpu_packet_row {
    uint64_t offset;        /* edgpu_out_desc.offset */
    uint32_t len;           /* edgpu_out_desc.len */
    uint32_t packet_id;     /* edgpu_out_desc.packet_id */
    int64_t  arrival;       /* fTimeArrived */
    uint32_t source;        /* blob slot in the last host batch, or EDGPU_NO_SOURCE */
    uint32_t _pad;
} edgpu_packet_row;
/* The sub-streams of the current copy pass that carry descriptors or are new outputs
 * (EDGPU_SUB_NEW: a host deriving per-tick state from new outputs sees every one), compacted and
 * in table order:
 * rows[i] is row q[i] of the pass's sub-stream table (edgpu_fanout_result.substreams), i <
 * min(*n_out, cap); *n_out counts all of them.  A host delivering a tick reads back only what it
 * writes -- at 2-ms ticks a few % of a 32k-row table.  `rows` / `q`: device memory
 * (EDGPU_PTR_DEVICE) or host memory (EDGPU_PTR_HOST; pinned buffers from edgpu_host_alloc are
 * stored into by the kernel over PCIe, others through a device copy).  Syncs. */
int  edgpu_fanout_active(edgpu_ctx* ctx, edgpu_substream_out* rows, uint32_t* q, uint32_t cap, uint32_t* n_out,
                         int kind);
/* The rows of SELECTED sub-streams of the current copy pass only: sel[2k] is a row of the
 * sub-stream table, sel[2k + 1] where its rows start in `rows`: rows[sel[2k + 1] + i] for its
 * descriptor desc_base + i, i < desc_count (rows at or past `nrows` are not written).  Two
 * EDGPU_SUB_IDENTITY sub-streams of one sender share their packets (the shorter a suffix of the
 * longer), so a host reads one sender's rows once for all of them -- at C2 the module's
 * readback falls from 28 B per write to 32 B per relayed packet.  `sel` is host
 * memory; `rows` host (EDGPU_PTR_HOST) or device (EDGPU_PTR_DEVICE).  Serial ticks; syncs. */
int  edgpu_fanout_rows(edgpu_ctx* ctx, const uint32_t* sel, uint32_t nsel, edgpu_packet_row* rows, uint64_t nrows,
                       int ptr_kind);

/* Packs regions of a fan-out arena (16-B aligned offsets and lengths; in the order given)
 * back to back into `dst` on the context stream -- so a host egress brings only the distinct
 * bytes of a tick over PCIe instead of the whole write-many arena.  `dst` is device memory, or
 * pinned host memory from edgpu_host_alloc: the gather kernel then stores straight over PCIe
 * (one pass, ~53 GB/s on the MI355X box against ~29 GB/s for a DMA copy).
 * Synchronous: the bytes are in `dst` when the call returns. */
typedef struct edgpu_region {
    uint64_t offset;        /* arena byte offset, multiple of 16 */
    uint64_t bytes;         /* multiple of 16 */
} edgpu_region;
int  edgpu_arena_gather(edgpu_ctx* ctx, const edgpu_fanout_result* r, const edgpu_region* regions, uint32_t n,
                        void* dst, uint64_t dst_cap);

/* Name of the fan-out copy kernel of this context's last edgpu_fanout (before the first: the one
 * it would launch), for measurement reports.  Unless EDGPU_FANOUT selects one, a tick takes the
 * 32-packet-chunk kernel when any active sub-stream is RTSP-interleaved or rewrites (a per-output
 * patch) or when the outputs added since the last tick hold a quarter or more of its sub-stream
 * rows and at least 4096 of them (a join burst), else the 16-packet-chunk one; see DESIGN.md §3. */
const char* edgpu_fanout_kernel(edgpu_ctx* ctx);

/* Cumulative counters since context creation (syncs).  fanout_in_bytes counts the
 * ingested bytes the fan-out read (each referenced packet once per launch). */
typedef struct edgpu_counters {
    uint64_t relayed_packets;
    uint64_t relayed_bytes;
    uint64_t fanout_in_bytes;
    uint64_t fanout_launches;
    uint64_t ingested_packets;
    uint64_t ingested_bytes;
    uint64_t fanout_passes;     /* copy passes launched (> fanout_launches: over-capacity ticks) */
    uint64_t lost_passes;       /* passes a tick still owed when the next tick was planned */
    uint32_t senders;           /* sender rows (2 per track) and sub-stream rows of the tables: */
    uint32_t substream_rows;    /* removed sessions' / subscribers' rows are reused, best fit */
    uint64_t ring_grows;        /* sender rings grown so far (edgpu_config.ring_growth) */
    uint64_t ring_bytes;        /* device bytes of every live sender's two rings now */
    uint64_t ring_pool_bytes;   /* device bytes the ring pool holds now: live rings, rings on its free
                                   lists (reused by later sessions / growths) and unused chunk space */
    uint64_t ring_grow_failures; /* growths skipped because the device memory could not hold the new
                                    rings (growth is best effort; the ingest goes on) */
    uint64_t watchdog_timeouts; /* waits the GPU watchdog ended (edgpu_config.watchdog_ms) */
    uint64_t kernel_launches;   /* kernels the context's calls launched */
    uint64_t host_syncs;        /* times a call waited for the GPU (stream / event synchronize) */
} edgpu_counters;
int  edgpu_counters_get(edgpu_ctx* ctx, edgpu_counters* out);

/* Per-launch device durations (ms, HIP events on the ctx stream) recorded since the last
 * call, oldest first, for `which` = 0 fan-out copy kernel, 1 whole fan-out tick (plan +
 * copy), 2 ingest (with the keyframe index it carries), 3 keyframe index (no entries since the
 * index runs inside the ingest kernel).  Up to 256 launches are kept; the history is cleared
 * after reading.  Syncs. */
int  edgpu_kernel_times(edgpu_ctx* ctx, int which, float* out_ms, uint32_t max_n, uint32_t* out_n);

/* Which per-launch timing events the context records from now on (default EDGPU_TIMING_ALL).
 * Every event is a marker the stream waits on between two kernels (4-8 us of idle GPU each on
 * MI355X, profiles/r03ak_timing_events_ab/): EDGPU_TIMING_FANOUT keeps only the fan-out copy
 * kernel's pair (edgpu_kernel_times which = 0), EDGPU_TIMING_NONE records none.  Rings not
 * recorded return no entries; edgpu_last_timings reports their last recorded pair, or 0. */
#define EDGPU_TIMING_NONE    0
#define EDGPU_TIMING_FANOUT  1
#define EDGPU_TIMING_ALL     2
int  edgpu_set_timing(edgpu_ctx* ctx, int level);

/* Copies device memory of this context to the host (synchronous).  Reads of 256 KiB or more
 * into pinned memory from edgpu_host_alloc are done by a copy kernel storing over PCIe (faster
 * than the DMA engine's device-to-host copy here); other reads are hipMemcpy copies. */
int  edgpu_copy_to_host(edgpu_ctx* ctx, void* dst, const void* device_src, uint64_t bytes);

/* Device-side timing of the last edgpu_fanout's kernels (HIP events on the ctx stream),
 * in milliseconds: [0] fan-out copy kernel, [1] whole fan-out (plan + copy),
 * [2] ingest (with the keyframe index), [3] 0 (the index runs inside the ingest). */
int  edgpu_last_timings(edgpu_ctx* ctx, float out_ms[4]);

/* Keyframe fast start: bytes a joining subscriber of `session`/`track` would receive now
 * (key pointer -> newest), cf. CKeyFrameCache (CommonUtilitiesLib/keyframecache.h:14-72). */
int  edgpu_gop_span(edgpu_ctx* ctx, uint32_t session, uint32_t track,
                    uint64_t* out_packets, uint64_t* out_bytes);

/* Copies the GOP a joining subscriber of `session`/`track` would receive (key pointer ->
 * newest, RTP sender) to host memory in CKeyFrameCache's TLV record format
 * [0x28][BE16 len][packet][0x29] (CommonUtilitiesLib/keyframecache.cpp:103-143), so the
 * keyframecache interface is served from the GPU's GOP index.  Empty packets (SSRC-filtered)
 * are skipped.  Returns EDGPU_OUT_OVERFLOW if `cap` is too small.  Syncs. */
int  edgpu_gop_copy(edgpu_ctx* ctx, uint32_t session, uint32_t track, uint8_t* dst, uint64_t cap,
                    uint64_t* out_len, uint32_t* out_packets);

/* ---- Cross-GPU keyframe fast start (BASELINE config C4) ----
 * Streams are owned by one GPU (FNV-1a-64 of the stream ID); a subscriber whose egress GPU
 * differs joins a *replica session* there.  The owner exports a session image -- the part
 * of each sender ring a new output can still be served from: key pointer -> newest, or the
 * new-output window when there is no key (ReflectorStream.cpp:1058-1069, 1201-1231) --
 * which travels once per (session, destination GPU) over xGMI (edgpu_memcpy_peer inside a
 * process, RCCL send/recv between processes), and the replica imports it.  A subscriber
 * joining the replica then receives exactly what it would have received joining the owner.
 * Later ticks ship delta images (packets after the previous export's heads), so a replica
 * follows its owner without re-sending the GOP.  Replica sessions are created with
 * edgpu_session_add from the owner's SDP and are never passed to edgpu_ingest.
 *
 * Image format (16-B aligned sections): 64-B header {magic "EDGI", version 1, ntracks,
 * nsenders, bytes, export time, session video-key flag, delta}, per track the packet-id
 * counter, per sender its ring state, then per sender the packet metadata (32 B each) and
 * the slot bytes ('$' 0 BE16(len) + packet + pad) of the packets carried. */
#define EDGPU_IMAGE_FULL 0xFFFFFFFFFFFFFFFFull

/* Exports images of `sessions[0..n)` into device memory `dst` (capacity `cap`), image i
 * at dst + offsets[i], offsets[n] = total bytes.  `from` is NULL (full images) or holds, per
 * sender of each listed session in order (2 * ntracks per session: track t RTP = 2t,
 * RTCP = 2t+1), EDGPU_IMAGE_FULL or the first queue index of a delta (a previous call's
 * `heads` value).  `heads` (optional, same shape) receives each sender's newest index + 1.
 * With dst == NULL only offsets/heads are computed (size query).  Syncs. */
int  edgpu_session_export(edgpu_ctx* ctx, const uint32_t* sessions, uint32_t n, int64_t now_ms,
                          const uint64_t* from, void* dst, uint64_t cap, uint64_t* offsets,
                          uint64_t* heads);

/* Applies images (device memory readable by this context's GPU; offsets as returned by the
 * export, n + 1 entries) to replica sessions `sessions[0..n)` of this context.  A delta
 * must start at the replica's current head.  Returns EDGPU_BAD_ARGUMENT for a mismatched
 * or out-of-order image, EDGPU_RING_OVERFLOW if the replica's rings are too small.  Syncs. */
int  edgpu_session_import(edgpu_ctx* ctx, const void* images, const uint64_t* offsets, uint32_t n,
                          const uint32_t* sessions);
/* Replica feedback (Q9 on a replica).  A backpressure report that relocates an output's bookmark
 * to the newest key frame sets the session's video-key-update flag
 * (ReflectorSender::NeedRelocateBookMark -> ReflectorSession::SetHasVideoKeyFrameUpdate(true),
 * ReflectorStream.cpp:1311-1317), and the session's next audio packet becomes the audio key
 * pointer (:1913-1930).  A replica session does not ingest: its relocations must reach the owner
 * before the owner's next edgpu_keyframe_index.  edgpu_session_relocations: out[i] = 1 when a
 * relocation happened on sessions[i] (of this context) since the last call; the indication is
 * cleared.  edgpu_session_key_update: sets the flag on the owner's sessions (not while an ingest
 * awaits its keyframe index). */
int  edgpu_session_relocations(edgpu_ctx* ctx, const uint32_t* sessions, uint32_t n, uint8_t* out);
int  edgpu_session_key_update(edgpu_ctx* ctx, const uint32_t* sessions, uint32_t n);

/* Enqueues a device-to-device copy from GPU `src_device` into this context's GPU on the
 * context stream (hipMemcpyPeerAsync over xGMI; a plain device copy when the devices are
 * the same).  Stream-ordered before the next call on this context. */
int  edgpu_memcpy_peer(edgpu_ctx* ctx, void* dst, int src_device, const void* src, uint64_t bytes);

/* Device memory on this context's GPU for image buffers (hipMalloc / hipFree).  Peer access
 * to it is enabled for every GPU that can reach this one, so RCCL and peer copies may use it. */
int  edgpu_device_alloc(edgpu_ctx* ctx, uint64_t bytes, void** out);
int  edgpu_device_free(edgpu_ctx* ctx, void* ptr);

/* Peer mailboxes between processes (one process per GPU): the steady-state replica feed without a
 * collective (easydarwin_amd/replica.py PeerMailbox).  edgpu_ipc_export gives the
 * handle of a buffer from edgpu_device_alloc (hipIpcGetMemHandle, HSA dmabuf IPC); another process
 * opens it with edgpu_ipc_open and gets a pointer its own GPU reads and writes over xGMI (peer
 * access enabled lazily) -- edgpu_session_import can read images straight from it, and
 * edgpu_copy_to_host / edgpu_copy_to_device move its header words.  edgpu_ipc_close unmaps it. */
#define EDGPU_IPC_HANDLE_BYTES 64
int  edgpu_ipc_export(edgpu_ctx* ctx, const void* device_ptr, uint8_t handle[EDGPU_IPC_HANDLE_BYTES]);
int  edgpu_ipc_open(edgpu_ctx* ctx, const uint8_t handle[EDGPU_IPC_HANDLE_BYTES], void** out);
int  edgpu_ipc_close(edgpu_ctx* ctx, void* ptr);
/* Copies host memory into device memory this context's GPU can write (its own, or a peer buffer
 * from edgpu_ipc_open); complete when the call returns. */
int  edgpu_copy_to_device(edgpu_ctx* ctx, void* device_dst, const void* src, uint64_t bytes);
/* Diagnostics: enqueues on the context stream one wave that waits `us` microseconds of the device
 * clock and exits -- work the GPU watchdog (edgpu_config.watchdog_ms) can time out on. */
int  edgpu_debug_stall(edgpu_ctx* ctx, uint32_t us);
/* The host CPUs of device `device`'s NUMA node (the sysfs local_cpulist of its PCI function) that
 * the calling thread may run on: cpus[0 .. min(*n_out, cap)), *n_out = how many -- where a server
 * hosting the module belongs (tools/bench_module.py --affinity gpu-node).  No
 * reference counterpart (host placement next to the GPU). */
int  edgpu_device_local_cpus(int device, uint32_t* cpus, uint32_t cap, uint32_t* n_out);

#ifdef __cplusplus
}
#endif
#endif /* EDGPU_H */
