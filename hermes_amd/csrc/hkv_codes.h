// hkv_codes.h -- protocol codes and byte offsets shared by host and device code.
// Codes restate include/hermes/spacetime.h:32-121; offsets are the reference's gcc layouts
// (see hermes_amd/layout.py for the per-field table).
#pragma once
#include <stdint.h>

namespace hkv {

enum : uint8_t {  // hermes_states_t, spacetime.h:42-48
    kValid = 1, kInvalid = 2, kInvalidWrite = 3, kWrite = 4, kReplay = 5
};
enum : uint8_t {  // input opcodes, spacetime.h:51-62
    kOpGet = 111, kOpPut = 112, kOpRmw = 113, kOpInv = 114, kOpAck = 115, kOpVal = 116,
    kOpCrd = 117, kOpMembChange = 118, kOpMembComplete = 119
};
enum : uint8_t {  // response opcodes, spacetime.h:65-89
    kGetComplete = 121, kPutSuccess = 122, kReplaySuccess = 123, kInvSuccess = 124,
    kAckSuccess = 125, kLastAckSuccess = 126, kLastAckNoBcast = 127, kPutComplete = 128,
    kValSuccess = 129, kMiss = 130, kGetStall = 131, kPutStall = 132,
    kPutCompleteSendVals = 133, kSendCrd = 134, kRmwSuccess = 135, kRmwStall = 136,
    kRmwComplete = 137, kRmwAbort = 138, kOpInvAbort = 139
};
enum : uint8_t {  // op bucket states, spacetime.h:95-106
    kEmpty = 140, kNew = 141, kComplete = 142, kInProgressPut = 143, kInProgressReplay = 144,
    kReplayComplete = 145, kInProgressGet = 146, kReplayCompleteSendVals = 147,
    kInProgressRmw = 148, kRmwCompleteSendVals = 149
};
enum : uint8_t { kInvOutOfGroup = 153 };  // spacetime.h:109-113
enum : int { kLocal = 0, kLocalAfterMemb = 1, kInvs = 2, kAcks = 3, kVals = 4 };

constexpr uint8_t kObiEmpty = 255;   // ST_OP_BUFFER_INDEX_EMPTY
constexpr uint8_t kLwidEmpty = 127;  // LAST_WRITER_ID_EMPTY
constexpr uint8_t kCidEmpty = 255;   // TIE_BREAKER_ID_EMPTY
constexpr int kOpMetaSize = 16;      // sizeof(spacetime_op_meta_t)
constexpr int kObjMetaSize = 15;     // sizeof(spacetime_object_meta)
constexpr int kEntryMetaOff = 18;    // mica key (16) + opcode + val_len
constexpr int kEntryValueOff = kEntryMetaOff + kObjMetaSize;  // 33
constexpr int kOpValueOff = 18;      // spacetime_op_t.value

// Runtime geometry of one table (one build variant of the reference).
struct Geometry {
    uint64_t bkt_mask;
    uint64_t log_cap;
    uint64_t log_mask;
    uint64_t log_head;      // final head after populate (wrap check, hermesKV.c:969-970)
    uint32_t entry_size;    // sizeof(struct mica_op): 64, or 320 with big objects
    uint32_t st_value;      // ST_VALUE_SIZE: 31 or 287
    uint32_t kvs_value;     // KVS_VALUE_SIZE: 46 or 302
    uint32_t shift;         // SHIFT_BITS
    uint32_t op_size;       // sizeof(spacetime_op_t)
    uint32_t entry_unit;    // divisor turning a physical log offset into a dense entry id
    uint32_t rmw_enabled;
    uint32_t machine_id;
    uint32_t skew;          // HKV_SKEW_* (hkv_config.skew_flags)
};
constexpr uint32_t kSkewReadComplete = 1u;   // ENABLE_READ_COMPLETE_AFTER_VAL_RECV_OF_HOT_REQS
constexpr uint32_t kSkewWriteCoalesce = 2u;  // ENABLE_WRITE_COALESCE_TO_THE_SAME_KEY_IN_SAME_NODE

}  // namespace hkv
