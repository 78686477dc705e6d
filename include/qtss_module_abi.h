/*
 * qtss_module_abi.h -- the QTSS module plugin ABI, restated for the MI355X reflector module
 * (libQTSSReflectorModule.so, easydarwin_amd/csrc/qtss_reflector_module.cpp).
 *
 * EasyDarwin (Darwin Streaming Server 5) loads a module by calling its main entry point
 * with a QTSS_PrivateArgs block; the module returns its dispatch function and from then on
 * the server calls it per role, while the module calls the server through a table of
 * callback function pointers.  This header restates exactly the part of that ABI the
 * reflector path uses -- same numeric values, same structure layouts -- so the engine's module
 * drops into an unmodified server.  Every item cites the reference declaration it mirrors
 * (paths relative to the EasyDarwin reference tree); tests/test_qtss_abi.py compiles this
 * header beside the reference headers and static_asserts every value, size and offset.
 *
 *   module entry / stub main      APIStubLib/QTSS_Private.cpp:44-59, QTSS.h:1271-1285
 *   QTSS_PrivateArgs              APIStubLib/QTSS_Private.h:130-138
 *   callback table indices        APIStubLib/QTSS_Private.h:52-122
 *   error codes                   APIStubLib/QTSS.h:61-85
 *   write / play / response flags APIStubLib/QTSS.h:105-124
 *   roles                         APIStubLib/QTSS.h:974-1028
 *   role parameter blocks         APIStubLib/QTSS.h:1073-1147, union :1223-1258
 *   QTSS_PacketStruct             APIStubLib/QTSS.h:1260-1265
 *   attribute ids used here       APIStubLib/QTSS.h:416-640
 *   RTSP methods                  RTSPUtilitiesLib/QTSSRTSPProtocol.h:43-63
 *
 * C++ only (the reflector module and its test server are C++); everything lives in
 * namespace edqtss so it can sit next to the reference headers in the layout test.
 */
#ifndef EDGPU_QTSS_MODULE_ABI_H
#define EDGPU_QTSS_MODULE_ABI_H

#include <stddef.h>
#include <stdint.h>

namespace edqtss {

constexpr uint32_t four_cc(char a, char b, char c, char d) {
    return (uint32_t)(uint8_t)a << 24 | (uint32_t)(uint8_t)b << 16 | (uint32_t)(uint8_t)c << 8 | (uint32_t)(uint8_t)d;
}

// QTSS_API_VERSION / QTSS_MAX_MODULE_NAME_LENGTH (macros in QTSS.h:41-42)
constexpr uint32_t kApiVersion = 0x00050000;
constexpr uint32_t kMaxModuleNameLength = 64;

typedef int32_t  QTSS_Error;
enum : int32_t {
    QTSS_NoErr = 0, QTSS_RequestFailed = -1, QTSS_Unimplemented = -2, QTSS_RequestArrived = -3,
    QTSS_OutOfState = -4, QTSS_NotAModule = -5, QTSS_WrongVersion = -6, QTSS_IllegalService = -7,
    QTSS_BadIndex = -8, QTSS_ValueNotFound = -9, QTSS_BadArgument = -10, QTSS_ReadOnly = -11,
    QTSS_NotPreemptiveSafe = -12, QTSS_NotEnoughSpace = -13, QTSS_WouldBlock = -14,
    QTSS_NotConnected = -15, QTSS_FileNotFound = -16, QTSS_NoMoreData = -17,
    QTSS_AttrDoesntExist = -18, QTSS_AttrNameExists = -19, QTSS_InstanceAttrsNotAllowed = -20,
};

typedef void*    QTSS_Object;
typedef void*    QTSS_StreamRef;
typedef int64_t  QTSS_TimeVal;
typedef uint32_t QTSS_AttributeID;
typedef uint32_t QTSS_ObjectType;
typedef uint32_t QTSS_Role;
typedef uint32_t QTSS_AttrDataType;
typedef uint32_t QTSS_RTSPMethod;
typedef uint32_t QTSS_RTPTransportType;
typedef uint32_t QTSS_RTPTransportMode;
typedef uint32_t QTSS_RTPSessionState;
typedef uint32_t QTSS_RTPPayloadType;
typedef uint32_t QTSS_CliSesClosingReason;

// QTSS_Write flags (QTSS.h:105-112), QTSS_Play flags (:97-101), response flags (:115-119)
enum : uint32_t {
    qtssWriteFlagsNoFlags = 0, qtssWriteFlagsIsRTP = 1, qtssWriteFlagsIsRTCP = 2,
    qtssWriteFlagsWriteBurstBegin = 4, qtssWriteFlagsBufferData = 8,
    qtssPlayFlagsSendRTCP = 0x10, qtssPlayFlagsAppendServerInfo = 0x20,
    qtssPlayRespWriteTrackInfo = 1, qtssSetupRespDontWriteSSRC = 2,
};

// transports, modes, states, payload types (QTSS.h:149-259)
enum : uint32_t {
    qtssPausedState = 0, qtssPlayingState = 1,
    qtssRTPTransportTypeUDP = 0, qtssRTPTransportTypeTCP = 2,
    qtssRTPTransportModePlay = 0, qtssRTPTransportModeRecord = 1,
    qtssUnknownPayloadType = 0, qtssVideoPayloadType = 1, qtssAudioPayloadType = 2,
    qtssCliSesCloseClientTeardown = 0,
    qtssCliSesTearDownBroadcastEnded = 4,            // QTSS_CliSesTeardownReason (QTSS.h:174-180)
};

// RTSP methods (QTSSRTSPProtocol.h:43-63)
enum : uint32_t {
    qtssDescribeMethod = 0, qtssSetupMethod = 1, qtssTeardownMethod = 2, qtssPlayMethod = 3,
    qtssPauseMethod = 4, qtssOptionsMethod = 5, qtssAnnounceMethod = 6, qtssRecordMethod = 10,
};

// attribute data types (QTSS.h:358-378)
enum : uint32_t {
    qtssAttrDataTypeUnknown = 0, qtssAttrDataTypeCharArray = 1, qtssAttrDataTypeBool16 = 2,
    qtssAttrDataTypeUInt16 = 4, qtssAttrDataTypeSInt32 = 5, qtssAttrDataTypeUInt32 = 6, qtssAttrDataTypeVoidPointer = 13,
};

// object types (QTSS.h:266-282)
enum : uint32_t {
    qtssRTPStreamObjectType = four_cc('r', 's', 't', 'o'),
    qtssClientSessionObjectType = four_cc('c', 's', 'e', 'o'),
    qtssRTSPSessionObjectType = four_cc('s', 's', 'e', 'o'),
    qtssRTSPRequestObjectType = four_cc('s', 'r', 'q', 'o'),
    qtssTextMessagesObjectType = four_cc('t', 'x', 't', 'o'),
    qtssModulePrefsObjectType = four_cc('m', 'o', 'd', 'p'),
    qtssPrefsObjectType = four_cc('p', 'r', 'f', 'o'),
    qtssModuleObjectType = four_cc('m', 'o', 'd', 'o'),
    qtssAttrInfoObjectType = four_cc('a', 't', 't', 'r'),
    qtssUserProfileObjectType = four_cc('u', 's', 'p', 'o'),
};

// request actions (QTSS.h:127-131), auth schemes (:195-197), RTSP status codes
// (QTSSRTSPProtocol.h:146-186: an index, the wire code in the comment)
enum : uint32_t {
    qtssActionFlagsNoFlags = 0, qtssActionFlagsRead = 1, qtssActionFlagsWrite = 2,
    qtssAuthNone = 0, qtssAuthBasic = 1, qtssAuthDigest = 2,
};
enum : uint32_t {
    qtssSuccessOK = 1,              // 200
    qtssClientBadRequest = 13,      // 400
    qtssClientUnAuthorized = 14,    // 401
    qtssClientForbidden = 16,       // 403
    qtssClientNotFound = 17,        // 404
    qtssPreconditionFailed = 25,    // 412
    qtssServerUnavailable = 44,     // 503
};

// attribute ids read or written by the reflector module
enum : uint32_t {
    // RTP stream object (QTSS.h:416-453)
    qtssRTPStrTrackID = 0, qtssRTPStrPayloadName = 2, qtssRTPStrPayloadType = 3,
    qtssRTPStrFirstSeqNumber = 4, qtssRTPStrFirstTimestamp = 5, qtssRTPStrTimescale = 6,
    qtssRTPStrTransportType = 31,
    // client session object (QTSS.h:473-512)
    qtssCliSesStreamObjects = 0, qtssCliSesState = 7, qtssCliSesFirstUserAgent = 9,
    qtssCliTeardownReason = 23, qtssCliSesTimeoutMsec = 32, qtssCliSesOverBufferEnabled = 33,
    // module object (QTSS.h:894-905), attribute-info object (:911-918), server prefs (:718-800)
    qtssModPrefs = 4, qtssAttrName = 0, qtssAttrID = 1, qtssAttrDataType = 2,
    qtssPrefsMovieFolder = 5, qtssPrefsPlayersReqRTPHeader = 70,
    // RTSP request object (QTSS.h:588-623)
    qtssRTSPReqFilePath = 2, qtssRTSPReqFileName = 5, qtssRTSPReqFileDigit = 6,
    qtssRTSPReqMethod = 9, qtssRTSPReqRespKeepAlive = 13, qtssRTSPReqQueryString = 23,
    qtssRTSPReqContentLen = 25, qtssRTSPReqTransportType = 28, qtssRTSPReqTransportMode = 29,
    qtssRTSPReqRootDir = 14,
    qtssRTSPReqSetUpServerPort = 30,                 // UInt16: server_port of a push SETUP's response
    qtssRTSPReqFilePathTrunc = 4, qtssRTSPReqStatusCode = 10, qtssRTSPReqUserAllowed = 19,
    qtssRTSPReqURLRealm = 20, qtssRTSPReqLocalPath = 21, qtssRTSPReqRespMsg = 24, qtssRTSPReqAction = 31,
    qtssRTSPReqUserProfile = 32, qtssRTSPReqAuthScheme = 34, qtssRTSPReqUserFound = 39, qtssRTSPReqAuthHandled = 40,
    // RTSP session object (QTSS.h:528-546)
    qtssRTSPSesRemoteAddrStr = 5,
    // user profile object (QTSS.h:928-935)
    qtssUserName = 0, qtssUserGroups = 2, qtssUserRealm = 3,
};

// RTSP header ids (QTSSRTSPProtocol.h:68-100)
enum : uint32_t { qtssCacheControlHeader = 11, qtssContentLengthHeader = 17 };

// roles (QTSS.h:974-1028)
enum : uint32_t {
    QTSS_Register_Role = four_cc('r', 'e', 'g', ' '),
    QTSS_Initialize_Role = four_cc('i', 'n', 'i', 't'),
    QTSS_Shutdown_Role = four_cc('s', 'h', 'u', 't'),
    QTSS_RereadPrefs_Role = four_cc('p', 'r', 'e', 'f'),
    QTSS_Interval_Role = four_cc('t', 'i', 'm', 'r'),
    QTSS_RTSPRoute_Role = four_cc('r', 'o', 'u', 't'),
    QTSS_RTSPAuthorize_Role = four_cc('a', 'u', 't', 'h'),
    QTSS_RTSPPreProcessor_Role = four_cc('p', 'r', 'e', 'p'),
    QTSS_RTSPIncomingData_Role = four_cc('i', 'c', 'm', 'd'),
    QTSS_ClientSessionClosing_Role = four_cc('d', 'e', 's', 's'),
};

// role parameter blocks (QTSS.h:1073-1147)
struct QTSS_Register_Params {
    char outModuleName[kMaxModuleNameLength];
};
struct QTSS_Initialize_Params {
    QTSS_Object inServer;
    QTSS_Object inPrefs;
    QTSS_Object inMessages;
    QTSS_StreamRef inErrorLogStream;
    QTSS_Object inModule;
};
struct QTSS_StandardRTSP_Params {
    QTSS_Object inRTSPSession;
    QTSS_Object inRTSPRequest;
    QTSS_Object inRTSPHeaders;
    QTSS_Object inClientSession;
};
struct QTSS_IncomingData_Params {
    QTSS_Object inRTSPSession;
    QTSS_Object inClientSession;
    char* inPacketData;
    uint32_t inPacketLen;
};
struct QTSS_ClientSessionClosing_Params {
    QTSS_Object inClientSession;
    QTSS_CliSesClosingReason inReason;
};
// The server passes a pointer to its QTSS_RoleParams union (QTSS.h:1223-1258); every member
// starts at offset 0, so the module reads the one block of the role being dispatched.
union QTSS_RoleParams {
    QTSS_Register_Params regParams;
    QTSS_Initialize_Params initParams;
    QTSS_StandardRTSP_Params rtspRequestParams;
    QTSS_IncomingData_Params rtspIncomingDataParams;
    QTSS_ClientSessionClosing_Params clientSessionClosingParams;
};

// QTSS_Write's packet for an RTP stream object (QTSS.h:1260-1265)
struct QTSS_PacketStruct {
    void* packetData;
    QTSS_TimeVal packetTransmitTime;
    QTSS_TimeVal suggestedWakeupTime;
};

// callback table (QTSS_Private.h:49-127)
typedef QTSS_Error (*QTSS_CallbackProcPtr)(...);
typedef QTSS_Error (*QTSS_DispatchFuncPtr)(QTSS_Role inRole, QTSS_RoleParams* inParams);
enum : uint32_t {
    kMillisecondsCallback = 2, kAddRoleCallback = 4, kIDForTagCallback = 6,
    kGetAttributePtrByIDCallback = 7, kGetAttributeByIDCallback = 8, kSetAttributeByIDCallback = 9,
    kWriteCallback = 10, kAppendRTSPHeadersCallback = 17, kSendStandardRTSPCallback = 18,
    kAddRTPStreamCallback = 19, kPlayCallback = 20, kPauseCallback = 21, kTeardownCallback = 22,
    kRequestEventCallback = 23, kSetIdleTimerCallback = 24, kReadCallback = 27,
    kSendRTSPHeadersCallback = 16, kOpenFileObjectCallback = 25, kCloseFileObjectCallback = 26,
    kGetNumValuesCallback = 30, kAddStaticAttributeCallback = 35, kAddInstanceAttributeCallback = 36,
    kGetAttrInfoByNameCallback = 39, kGetValueAsStringCallback = 41, kValueToStringCallback = 45,
    kRemoveValueCallback = 46, kRefreshTimeOutCallback = 52, kLockObjectCallback = 55, kUnlockObjectCallback = 56,
    kLastCallback = 62,
};
struct QTSS_Callbacks {
    QTSS_CallbackProcPtr addr[kLastCallback];
};
struct QTSS_PrivateArgs {
    uint32_t inServerAPIVersion;
    QTSS_Callbacks* inCallbacks;
    QTSS_StreamRef inErrorLogStream;
    uint32_t outStubLibraryVersion;
    QTSS_DispatchFuncPtr outDispatchFunction;
};

}  // namespace edqtss

extern "C" {
/* The module's main entry point, the symbol the server resolves for a dynamic or
 * compiled-in reflector module (QTSSReflectorModule.cpp:228-231). */
edqtss::QTSS_Error QTSSReflectorModule_Main(void* inPrivateArgs);

/* Engine extension: runs one reflect tick (ingest of everything pushed since the last tick,
 * keyframe index, fan-out, QTSS_Write of every send-ready packet) at QTSS_Milliseconds().
 * The module's own tick thread calls it every `edgpu_tick_msec` (module pref, default 20 ms);
 * with the pref `edgpu_manual_tick` (or EDGPU_QTSS_MANUAL_TICK=1) the host calls it instead.
 * It stands in for the ReflectorSocket tasks that run ReflectPackets in the reference
 * (ReflectorStream.cpp:1676-1714).  Returns a QTSS_Error. */
edqtss::QTSS_Error EDGPU_QTSSReflectorModule_Tick(void);

/* Engine extension, manual mode: reads every datagram waiting on the UDP push sockets now (the
 * reader thread's work, ReflectorSocket::GetIncomingData, ReflectorStream.cpp:1716-1735);
 * returns how many were handed to the engine. */
uint32_t EDGPU_QTSSReflectorModule_PollUDP(void);

/* Engine extension: measurements of the last tick (tools/qtss_replay --bench).  hold_ms is how
 * long the tick held the module's session lock (RTSP roles wait that long; the pushers' ingest
 * never does); readback_bytes is what crossed PCIe back (the tick's distinct bytes, descriptors
 * and sub-stream table) against arena_bytes, the write-many output on the GPU. */
typedef struct EDGPU_QTSSTickInfo {
    uint64_t ingested_packets, ingested_bytes;
    uint64_t readback_bytes, arena_bytes;
    uint64_t writes;                    /* QTSS_Write calls */
    double   ingest_ms, fanout_ms, readback_ms, write_ms, hold_ms;
    uint64_t ticks, failed_ticks;       /* since Initialize */
    int64_t  last_error;                /* the engine's code of the newest failed tick, or 0 */
    uint64_t prestaged_bytes;           /* of the tick's batch, copied to the device while it filled */
    uint64_t passes;                    /* copy passes of the tick (> 1: it exceeded the arena) */
    uint64_t rereads;                   /* RereadPrefs calls handled since Initialize */
    double   hold_max_ms, hold_sum_ms;  /* the longest lock hold of any tick / the sum of all, since
                                           Initialize (RTSP roles wait behind a tick) */
    uint64_t stream_errors;             /* sessions a tick marked since Initialize: a sender ring lost
                                           a packet one of their outputs needed (logged by name;
                                           the ticks went on for every other session) */
    /* sums over every tick since Initialize (a host takes differences over a window): wall time
       (start to the last write), then its ingest / fan-out / readback / write parts */
    double   wall_sum_ms, ingest_sum_ms, fanout_sum_ms, readback_sum_ms, write_sum_ms;
} EDGPU_QTSSTickInfo;
edqtss::QTSS_Error EDGPU_QTSSReflectorModule_LastTick(EDGPU_QTSSTickInfo* out);
}

#endif /* EDGPU_QTSS_MODULE_ABI_H */
