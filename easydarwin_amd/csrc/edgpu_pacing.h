// edgpu_pacing.h -- the server's write gate for the engine's own socket egress (Q20; edgpu_egress
// with edgpu_egress_pacing).  Host code.
//
// Behind the reference module, every relayed packet reaches the server's RTPStream::Write
// (Server.tproj/RTPStream.cpp:1048-1147) as a QTSS_PacketStruct whose transmit time
// RTPSessionOutput::WritePacket computed (RTPSessionOutput.cpp:603-608).  Before the socket, the
// server (1) asks the session's over-buffer window whether the packet may go now
// (RTPOverbufferWindow::CheckTransmitTime, RTPOverbufferWindow.cpp:68-147; RTP always, RTCP when
// overbuffering is off) -- QTSS_WouldBlock if not, which stops the output for this reflect and, on a
// new output's first pass, makes the packet's age the output's buffer delay (RTPSessionOutput.cpp:
// 612-622); (2) for RTP of a TCP non-video stream runs RTPStream::UpdateQualityLevel
// (RTPStream.cpp:936-1045), which drops a packet that has fallen too far behind; (3) after a
// written RTP packet adds it to the window (:1208-1213).  This is that gate, restated for the
// egress: the window class is pinned against the compiled reference (tests/test_pacing.py), the
// whole gate against the reference harness's server gate (tests/test_gpu_egress.py).
#pragma once
#include <cstdint>
#include <vector>

namespace edpace {

// The server prefs the gate reads (QTSServerPrefs.cpp defaults) and the reflector's own
// (ReflectorStream::Initialize prefs, ReflectorStream.cpp:87-117).
struct Config {
    int64_t bucket_delay_ms = 73;       // reflector_bucket_offset_delay_msec (sBucketDelayInMsec)
    uint32_t bucket_size = 16;          // ReflectorStream::sBucketSize
    int64_t over_buffer_ms = 1000;      // reflector_buffer_size_sec x 1000: a new output's buffer delay
    uint32_t send_interval_ms = 50;     // send_interval
    uint32_t max_send_ahead_s = 25;     // max_send_ahead_time
    float overbuffer_rate = 2.0f;       // overbuffer_rate
    // SetThinningParams (RTPStream.cpp:897-918) with the default 1.5-s late tolerance (no adjustment)
    int64_t drop_all_packets_ms = 2500; // drop_all_packets_delay (non-video streams)
    int64_t thin_all_the_way_ms = 1500; // thin_all_the_way_delay
    int64_t start_thinning_ms = 0;      // start_thinning_delay
};

// RTPOverbufferWindow (RTPOverbufferWindow.cpp:36-178), one per RTP session: the same fields,
// types and arithmetic.
class OverbufferWindow {
public:
    OverbufferWindow(uint32_t sendInterval, uint32_t initialWindowSize, uint32_t maxSendAheadSecs, float rate)
        : fWindowSize((int32_t)initialWindowSize), fSendInterval((int32_t)sendInterval),
          fMaxSendAheadTime(maxSendAheadSecs * 1000), fOverbufferRate(rate) {
        if (fSendInterval == 0) {
            fOverbufferingEnabled = false;
            fSendInterval = 200;
        }
        if (fOverbufferRate < 1.0) fOverbufferRate = 1.0;
    }
    // -1: send now; else the time the packet may go (the caller returns QTSS_WouldBlock when it is
    // later than now)
    int64_t CheckTransmitTime(int64_t transmit, int64_t now, int32_t size) {
        if (now - fBucketBegin > fSendInterval) {
            fPreviousBucketBegin = fBucketBegin;
            fBucketBegin = now;
            if (fPreviousBucketBegin == 0) fPreviousBucketBegin = fBucketBegin - fSendInterval;
            fBytesDuringBucket = 0;
            if (now - fLastSecondStart > 1000) {
                fBytesDuringPreviousSecond = fBytesDuringLastSecond;
                fBytesDuringLastSecond = 0;
                fPreviousSecondStart = fLastSecondStart;
                fLastSecondStart = now;
            }
            fPreviousBucketTimeAhead = fBucketTimeAhead;
        }
        if (fOverbufferWindowBegin == -1) fOverbufferWindowBegin = now;
        if (transmit <= now + fSendInterval ||
            (fOverbufferingEnabled && transmit <= now + fSendInterval + (int64_t)fSendAheadDurationInMsec))
            return -1;
        if (!fOverbufferingEnabled || fWindowSize == 0) return transmit;
        if (fWindowSize != -1 && size * 5 > fWindowSize - fBytesSentSinceLastReport) return now + (int64_t)fSendInterval * 5;
        if (transmit - now > (int64_t)fMaxSendAheadTime) return transmit - (int64_t)fMaxSendAheadTime + fSendInterval;
        fBucketTimeAhead = transmit - now;
        if (fBucketTimeAhead < fPreviousBucketTimeAhead) return -1;
        const double ahead = (double)(now - fPreviousBucketBegin) * ((double)fOverbufferRate - 1.0);
        if ((double)(fBucketTimeAhead - fPreviousBucketTimeAhead) > ahead) {
            fBucketTimeAhead = fPreviousBucketTimeAhead + (int64_t)ahead;
            return now + fSendInterval;
        }
        return -1;
    }
    void AddPacketToWindow(int32_t size) {
        fBytesDuringBucket += size;
        fBytesDuringLastSecond += size;
        fBytesSentSinceLastReport += size;
    }
    void SetWindowSize(uint32_t bytes) { fWindowSize = (int32_t)bytes; fBytesSentSinceLastReport = 0; }
    void ResetOverBufferWindow() {
        fBytesDuringLastSecond = 0; fLastSecondStart = -1; fBytesDuringPreviousSecond = 0; fPreviousSecondStart = -1;
        fBytesDuringBucket = 0; fBucketBegin = 0; fBucketTimeAhead = 0; fPreviousBucketTimeAhead = 0;
        fOverbufferWindowBegin = -1;
    }
    void TurnOffOverbuffering() { fOverbufferingEnabled = false; }
    void TurnOnOverbuffering() { fOverbufferingEnabled = true; }
    bool OverbufferingEnabled() const { return fOverbufferingEnabled; }

private:
    int32_t fWindowSize;
    int32_t fBytesSentSinceLastReport = 0;
    int32_t fSendInterval;
    int32_t fBytesDuringLastSecond = 0;
    int64_t fLastSecondStart = -1;
    int32_t fBytesDuringPreviousSecond = 0;
    int64_t fPreviousSecondStart = -1;
    int32_t fBytesDuringBucket = 0;
    int64_t fBucketBegin = 0;
    int64_t fPreviousBucketBegin = 0;
    int64_t fBucketTimeAhead = 0;
    int64_t fPreviousBucketTimeAhead = 0;
    uint32_t fMaxSendAheadTime;
    bool fOverbufferingEnabled = true;
    float fOverbufferRate;
    uint32_t fSendAheadDurationInMsec = 1000;
    int64_t fOverbufferWindowBegin = -1;
};

// One player (an RTPSession with its RTPSessionOutput): the window, the thinning state the
// session keeps for all its streams, and the output's buffer delay.
struct Player {
    Player(const Config& c, bool tcp, bool overbuffer)
        : win(c.send_interval_ms, 0xFFFFFFFFu, c.max_send_ahead_s, c.overbuffer_rate), buffer_delay_ms(c.over_buffer_ms) {
        // the reflector turns overbuffering off for a player without a dynamic-rate header
        // (QTSSReflectorModule.cpp:1772-1777); a TCP stream opens the window (RTPStream.cpp:466-469)
        if (!overbuffer) win.TurnOffOverbuffering();
        if (tcp) win.SetWindowSize(0xFFFFFFFFu);
    }
    OverbufferWindow win;
    int64_t buffer_delay_ms;            // RTPSessionOutput::fBufferDelayMSecs
    int64_t play_time_ms = 0;           // RTPSession::fPlayTime
    int64_t last_check = 0, last_check_media = 0;   // fLastQualityCheckTime / MediaTime (session)
    bool started_thinning = false;      // fStartedThinning (session)
    std::vector<int64_t> last_delay;    // per track: RTPStream::fLastCurrentPacketDelay
    uint64_t stale_dropped = 0;
};

// RTPSessionOutput::WritePacket's transmit time (RTPSessionOutput.cpp:603-608): now less the
// bucket's lateness, plus (while the output has a buffer delay) the delay left for this packet.
inline int64_t transmit_time(int64_t now, int64_t lateness, int64_t buffer_delay, int64_t arrival) {
    int64_t t = now - lateness;
    if (buffer_delay > 0) t += buffer_delay - (now - arrival);
    return t;
}

// RTPStream::UpdateQualityLevel (RTPStream.cpp:936-1045) for a reflected stream: false = the
// packet is stale, drop it.  The reflector sets two quality levels (ReflectorSession.h:152-154,
// QTSSReflectorModule.cpp:1786-1787), so past the drop test the function only moves the level
// (nothing the egress writes depends on it).
inline bool keep_packet(Player& p, uint32_t track, bool video, bool tcp, int64_t transmit, int64_t delay, int64_t now,
                        const Config& c) {
    if (transmit <= p.play_time_ms) return true;
    if (video || !tcp) return true;                         // (:946-954)
    if (p.last_delay.size() <= track) p.last_delay.resize(track + 1, 0);
    int64_t& last = p.last_delay[track];
    if (p.last_check == 0) {
        p.last_check = now; p.last_check_media = transmit; last = delay;
        return true;
    }
    if (!p.started_thinning) {
        if (delay > c.start_thinning_ms && delay - last < 250) {
            if (delay < last) last = delay;
            return true;
        }
        p.started_thinning = true;
    }
    if (p.last_check == 0 || delay > c.thin_all_the_way_ms) {
        p.last_check = now; p.last_check_media = transmit; last = delay;
        if (delay > c.thin_all_the_way_ms && delay > c.drop_all_packets_ms) {
            p.stale_dropped++;
            return false;
        }
    }
    return true;
}

}  // namespace edpace
