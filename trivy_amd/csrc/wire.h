// Protobuf (proto3 wire format) of types.Secret for client/server mode:
// trivy.common.Secret (rpc/common/service.proto:152-156) with its
// SecretFinding / Code / Line / Layer messages (service.proto:191-223).
#pragma once
#include <cstdint>
#include <deque>
#include <string>
#include <vector>

#include "report.h"
#include "scanner.h"

namespace tsg {

// proto.Marshal(ConvertToRPCSecrets([]ftypes.Secret{sec})[0]): the Secret
// message of one file.  layer_of_finding (optional) gives each finding's
// Layer (set by the applier); absent -> empty Layer messages, as an fs scan.
// Fails like proto.Marshal when a string is not valid UTF-8.
bool secret_to_proto(const Secret& sec, const std::vector<LayerRef>* layer_of_finding, std::string* out,
                     std::string* err);

// proto.Unmarshal + ConvertFromRPCSecrets of one Secret message.  Rules named
// by the findings are appended to `rules` (the findings point at them); each
// finding's Layer goes to `layers`.  Unknown fields are skipped.
bool secret_from_proto(const uint8_t* data, size_t len, std::deque<Rule>* rules, Secret* out,
                       std::vector<LayerRef>* layers, std::string* err);

}  // namespace tsg
