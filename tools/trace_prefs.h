// tools/trace_prefs.h -- the preferences of a trace (easydarwin_amd/trace.py, version 4), for the
// replay tools (adapter_replay, qtss_replay).  TEST INFRASTRUCTURE.
//
// A trace names the prefs it overrides as "name=value" lines; every other pref has the
// reference's default (trace.py PREF_DEFAULTS: ReflectorStream.cpp:53-59, QTSSReflectorModule.cpp:
// 100-166, the shipped easydarwin.xml's player list).  A PREFS event replaces the overrides.
#pragma once
#include <cstdint>
#include <cstdlib>
#include <map>
#include <string>
#include <vector>

namespace trace_prefs {

inline const std::vector<std::pair<std::string, std::string>>& defaults() {
    static const std::vector<std::pair<std::string, std::string>> d = {
        {"reflector_bucket_offset_delay_msec", "73"}, {"reflector_buffer_size_sec", "1"},
        {"rtp_reflector_threshold_msec", "2000"}, {"reflector_rtp_info_offset_msec", "500"},
        {"kill_clients_when_broadcast_stops", "false"}, {"use_one_SSRC_per_stream", "true"},
        {"timeout_stream_SSRC_secs", "30"}, {"disable_rtp_play_info", "false"},
        {"enable_player_compatibility", "true"}, {"force_rtp_info_sequence_and_time", "false"},
        {"player_requires_rtp_header_info", "Android,vlc"},
        {"enable_broadcast_announce", "true"}, {"enable_broadcast_push", "true"},
        {"allow_duplicate_broadcasts", "false"}, {"timeout_broadcaster_session_secs", "30"},
        {"reflector_use_in_packet_receive_time", "false"}, {"reflector_in_packet_max_receive_sec", "60"},
        {"allow_broadcasts", "true"}, {"authenticate_local_broadcast", "false"}, {"BroadcasterGroup", "broadcaster"},
        {"ip_allow_list", "127.0.0.*"}, {"redirect_broadcast_keyword", ""}, {"redirect_broadcasts_dir", ""},
        {"allow_non_sdp_urls", "true"},
    };
    return d;
}

// the module prefs whose values are strings (easydarwin.xml CharArray prefs); ip_allow_list is a
// LIST-PREF: its comma-separated entries are its values
inline bool is_list(const std::string& k) { return k == "ip_allow_list"; }
inline bool is_string(const std::string& k) {
    return is_list(k) || k == "BroadcasterGroup" || k == "redirect_broadcast_keyword" || k == "redirect_broadcasts_dir";
}

// the user agent of a JOIN's player (trace.py USER_AGENTS, by ua_flags bit 0)
inline const char* user_agent(uint8_t ua_flags) { return (ua_flags & 1) ? "vlc/3.0.8 LibVLC/3.0.8" : "EasyPlayer/1.0"; }

struct Prefs {
    std::map<std::string, std::string> over;            // the trace's overrides

    static Prefs parse(const uint8_t* b, uint32_t n) {
        Prefs p;
        const std::string s((const char*)b, n);
        for (size_t i = 0; i < s.size();) {
            size_t e = s.find('\n', i);
            if (e == std::string::npos) e = s.size();
            const std::string line = s.substr(i, e - i);
            const size_t q = line.find('=');
            if (q != std::string::npos) p.over[line.substr(0, q)] = line.substr(q + 1);
            i = e + 1;
        }
        return p;
    }
    std::string get(const std::string& k) const {
        auto it = over.find(k);
        if (it != over.end()) return it->second;
        for (const auto& d : defaults())
            if (d.first == k) return d.second;
        return std::string();
    }
    uint32_t u32(const std::string& k) const { return (uint32_t)strtoul(get(k).c_str(), nullptr, 10); }
    bool flag(const std::string& k) const { return get(k) == "true"; }
    std::vector<std::string> list(const std::string& k) const {
        std::vector<std::string> out;
        const std::string l = get(k);
        for (size_t i = 0; i <= l.size();) {
            size_t e = l.find(',', i);
            if (e == std::string::npos) e = l.size();
            out.push_back(l.substr(i, e - i));
            i = e + 1;
        }
        return out;
    }
    // DoPlay's rtpInfoEnabled (QTSSReflectorModule.cpp:1962-1969) for a JOIN's player
    bool rtp_info_player(uint8_t ua_flags) const {
        const std::string ua = user_agent(ua_flags);
        bool on = false;
        if (flag("enable_player_compatibility"))
            for (const std::string& x : list("player_requires_rtp_header_info"))
                if (x == "*" || ua.find(x) != std::string::npos) { on = true; break; }
        if (flag("force_rtp_info_sequence_and_time")) on = true;
        if (flag("disable_rtp_play_info")) on = false;
        return on;
    }
};

}  // namespace trace_prefs
