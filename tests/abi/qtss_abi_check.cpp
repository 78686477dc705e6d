// Compile-time check (tests/test_qtss_abi.py): include/qtss_module_abi.h against the
// reference's own QTSS headers -- every constant, size and field offset the reflector module
// relies on must be identical.  Test infrastructure; compiled with the reference include path.
#include <cstddef>
#include "QTSS.h"
#include "QTSS_Private.h"
#include "qtss_module_abi.h"

namespace E = edqtss;
#define SAME(x) static_assert((long long)E::x == (long long)(::x), #x)
#define SAME_SIZE(T) static_assert(sizeof(E::T) == sizeof(::T), "sizeof " #T)
#define SAME_OFF(T, f) static_assert(offsetof(E::T, f) == offsetof(::T, f), "offsetof " #T "." #f)

static_assert(E::kApiVersion == QTSS_API_VERSION, "QTSS_API_VERSION");
static_assert(E::kMaxModuleNameLength == QTSS_MAX_MODULE_NAME_LENGTH, "QTSS_MAX_MODULE_NAME_LENGTH");
SAME(QTSS_NoErr); SAME(QTSS_RequestFailed); SAME(QTSS_Unimplemented); SAME(QTSS_RequestArrived);
SAME(QTSS_OutOfState); SAME(QTSS_NotAModule); SAME(QTSS_WrongVersion); SAME(QTSS_IllegalService);
SAME(QTSS_BadIndex); SAME(QTSS_ValueNotFound); SAME(QTSS_BadArgument); SAME(QTSS_ReadOnly);
SAME(QTSS_NotPreemptiveSafe); SAME(QTSS_NotEnoughSpace); SAME(QTSS_WouldBlock); SAME(QTSS_NotConnected);
SAME(QTSS_FileNotFound); SAME(QTSS_NoMoreData); SAME(QTSS_AttrDoesntExist); SAME(QTSS_AttrNameExists);
SAME(QTSS_InstanceAttrsNotAllowed);
SAME(qtssWriteFlagsNoFlags); SAME(qtssWriteFlagsIsRTP); SAME(qtssWriteFlagsIsRTCP);
SAME(qtssWriteFlagsWriteBurstBegin); SAME(qtssWriteFlagsBufferData);
SAME(qtssPlayFlagsSendRTCP); SAME(qtssPlayFlagsAppendServerInfo);
SAME(qtssPlayRespWriteTrackInfo); SAME(qtssSetupRespDontWriteSSRC);
SAME(qtssPausedState); SAME(qtssPlayingState); SAME(qtssRTPTransportTypeUDP); SAME(qtssRTPTransportTypeTCP);
SAME(qtssRTPTransportModePlay); SAME(qtssRTPTransportModeRecord);
SAME(qtssUnknownPayloadType); SAME(qtssVideoPayloadType); SAME(qtssAudioPayloadType);
SAME(qtssCliSesCloseClientTeardown); SAME(qtssCliSesTearDownBroadcastEnded); SAME(qtssCliTeardownReason); SAME(qtssCliSesTimeoutMsec);
SAME(qtssDescribeMethod); SAME(qtssSetupMethod); SAME(qtssTeardownMethod); SAME(qtssPlayMethod);
SAME(qtssPauseMethod); SAME(qtssOptionsMethod); SAME(qtssAnnounceMethod); SAME(qtssRecordMethod);
SAME(qtssAttrDataTypeCharArray); SAME(qtssAttrDataTypeSInt32); SAME(qtssAttrDataTypeUInt16); SAME(qtssAttrDataTypeUInt32);
SAME(qtssAttrDataTypeVoidPointer); SAME(qtssAttrDataTypeBool16); SAME(qtssAttrDataTypeUnknown);
SAME(qtssPrefsObjectType); SAME(qtssModuleObjectType); SAME(qtssAttrInfoObjectType);
SAME(qtssCliSesOverBufferEnabled); SAME(qtssModPrefs); SAME(qtssAttrName); SAME(qtssAttrID); SAME(qtssAttrDataType);
SAME(qtssPrefsPlayersReqRTPHeader); SAME(qtssPrefsMovieFolder); SAME(qtssRTSPReqRootDir);
SAME(kAddInstanceAttributeCallback); SAME(kGetAttrInfoByNameCallback); SAME(kGetValueAsStringCallback);
SAME(qtssRTPStreamObjectType); SAME(qtssClientSessionObjectType); SAME(qtssRTSPSessionObjectType);
SAME(qtssRTSPRequestObjectType); SAME(qtssTextMessagesObjectType); SAME(qtssModulePrefsObjectType);
SAME(qtssRTPStrTrackID); SAME(qtssRTPStrPayloadName); SAME(qtssRTPStrPayloadType);
SAME(qtssRTPStrFirstSeqNumber); SAME(qtssRTPStrFirstTimestamp); SAME(qtssRTPStrTimescale);
SAME(qtssRTPStrTransportType); SAME(qtssCliSesStreamObjects); SAME(qtssCliSesState);
SAME(qtssCliSesFirstUserAgent); SAME(qtssRTSPReqFilePath); SAME(qtssRTSPReqFileName);
SAME(qtssRTSPReqFileDigit); SAME(qtssRTSPReqMethod); SAME(qtssRTSPReqRespKeepAlive);
SAME(qtssRTSPReqQueryString); SAME(qtssRTSPReqContentLen); SAME(qtssRTSPReqTransportType);
SAME(qtssRTSPReqTransportMode); SAME(qtssRTSPReqSetUpServerPort); SAME(qtssCacheControlHeader); SAME(qtssContentLengthHeader);
SAME(QTSS_Register_Role); SAME(QTSS_Initialize_Role); SAME(QTSS_Shutdown_Role); SAME(QTSS_RereadPrefs_Role);
SAME(QTSS_Interval_Role); SAME(QTSS_RTSPRoute_Role); SAME(QTSS_RTSPAuthorize_Role);
SAME(QTSS_RTSPPreProcessor_Role); SAME(QTSS_RTSPIncomingData_Role); SAME(QTSS_ClientSessionClosing_Role);
SAME(kMillisecondsCallback); SAME(kAddRoleCallback); SAME(kIDForTagCallback);
SAME(kGetAttributePtrByIDCallback); SAME(kGetAttributeByIDCallback); SAME(kSetAttributeByIDCallback);
SAME(kWriteCallback); SAME(kAppendRTSPHeadersCallback); SAME(kSendStandardRTSPCallback);
SAME(kAddRTPStreamCallback); SAME(kPlayCallback); SAME(kPauseCallback); SAME(kTeardownCallback);
SAME(kRequestEventCallback); SAME(kSetIdleTimerCallback); SAME(kReadCallback); SAME(kGetNumValuesCallback);
SAME(kAddStaticAttributeCallback); SAME(kRemoveValueCallback); SAME(kLastCallback);
SAME(kValueToStringCallback); SAME(kRefreshTimeOutCallback); SAME(kLockObjectCallback); SAME(kUnlockObjectCallback);
SAME(kSendRTSPHeadersCallback); SAME(kOpenFileObjectCallback); SAME(kCloseFileObjectCallback);
SAME(qtssUserProfileObjectType); SAME(qtssActionFlagsNoFlags); SAME(qtssActionFlagsRead); SAME(qtssActionFlagsWrite);
SAME(qtssAuthNone); SAME(qtssAuthBasic); SAME(qtssAuthDigest);
SAME(qtssSuccessOK); SAME(qtssClientBadRequest); SAME(qtssClientUnAuthorized); SAME(qtssClientForbidden);
SAME(qtssClientNotFound); SAME(qtssPreconditionFailed); SAME(qtssServerUnavailable);
SAME(qtssRTSPReqFilePathTrunc); SAME(qtssRTSPReqStatusCode); SAME(qtssRTSPReqUserAllowed); SAME(qtssRTSPReqURLRealm);
SAME(qtssRTSPReqLocalPath); SAME(qtssRTSPReqRespMsg); SAME(qtssRTSPReqAction); SAME(qtssRTSPReqUserProfile);
SAME(qtssRTSPReqAuthScheme); SAME(qtssRTSPReqUserFound); SAME(qtssRTSPReqAuthHandled); SAME(qtssRTSPSesRemoteAddrStr);
SAME(qtssUserName); SAME(qtssUserGroups); SAME(qtssUserRealm);

static_assert(sizeof(E::QTSS_Error) == sizeof(::QTSS_Error), "QTSS_Error");
static_assert(sizeof(E::QTSS_Role) == sizeof(::QTSS_Role), "QTSS_Role");
static_assert(sizeof(E::QTSS_AttributeID) == sizeof(::QTSS_AttributeID), "QTSS_AttributeID");
static_assert(sizeof(E::QTSS_TimeVal) == sizeof(::QTSS_TimeVal), "QTSS_TimeVal");
static_assert(sizeof(E::QTSS_RTSPMethod) == sizeof(::QTSS_RTSPMethod), "QTSS_RTSPMethod");
SAME_SIZE(QTSS_PacketStruct);
SAME_OFF(QTSS_PacketStruct, packetData); SAME_OFF(QTSS_PacketStruct, packetTransmitTime);
SAME_OFF(QTSS_PacketStruct, suggestedWakeupTime);
SAME_SIZE(QTSS_Register_Params); SAME_SIZE(QTSS_Initialize_Params); SAME_SIZE(QTSS_StandardRTSP_Params);
SAME_SIZE(QTSS_IncomingData_Params); SAME_SIZE(QTSS_ClientSessionClosing_Params);
SAME_OFF(QTSS_Initialize_Params, inServer); SAME_OFF(QTSS_Initialize_Params, inPrefs);
SAME_OFF(QTSS_Initialize_Params, inMessages); SAME_OFF(QTSS_Initialize_Params, inErrorLogStream);
SAME_OFF(QTSS_Initialize_Params, inModule);
SAME_OFF(QTSS_StandardRTSP_Params, inRTSPSession); SAME_OFF(QTSS_StandardRTSP_Params, inRTSPRequest);
SAME_OFF(QTSS_StandardRTSP_Params, inRTSPHeaders); SAME_OFF(QTSS_StandardRTSP_Params, inClientSession);
SAME_OFF(QTSS_IncomingData_Params, inRTSPSession); SAME_OFF(QTSS_IncomingData_Params, inClientSession);
SAME_OFF(QTSS_IncomingData_Params, inPacketData); SAME_OFF(QTSS_IncomingData_Params, inPacketLen);
SAME_OFF(QTSS_ClientSessionClosing_Params, inClientSession);
SAME_OFF(QTSS_ClientSessionClosing_Params, inReason);
SAME_SIZE(QTSS_Callbacks);
SAME_SIZE(QTSS_PrivateArgs);
SAME_OFF(QTSS_PrivateArgs, inServerAPIVersion); SAME_OFF(QTSS_PrivateArgs, inCallbacks);
SAME_OFF(QTSS_PrivateArgs, inErrorLogStream); SAME_OFF(QTSS_PrivateArgs, outStubLibraryVersion);
SAME_OFF(QTSS_PrivateArgs, outDispatchFunction);
// the union members the module reads sit at offset 0 of the server's QTSS_RoleParams
static_assert(offsetof(::QTSS_RoleParams, regParams) == 0 && offsetof(::QTSS_RoleParams, initParams) == 0 &&
              offsetof(::QTSS_RoleParams, rtspRequestParams) == 0 &&
              offsetof(::QTSS_RoleParams, rtspIncomingDataParams) == 0 &&
              offsetof(::QTSS_RoleParams, clientSessionClosingParams) == 0, "role params at offset 0");
static_assert(sizeof(E::QTSS_RoleParams) <= sizeof(::QTSS_RoleParams), "role params fit the server's union");

int main() { return 0; }
