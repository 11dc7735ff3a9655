// Everything between Scanner.Scan's types.Secret and the `trivy -f json`
// document for the secret scanner, restated on
// the host:
//   * AnalysisResult.Sort for secrets      pkg/fanal/analyzer/analyzer.go:224-235
//   * ApplyLayers' secret merge             pkg/fanal/applier/docker.go:134-146, 186-188, 297-325
//   * image-config secret merge             pkg/scanner/local/scan.go:487-496
//   * secretsToResults                      pkg/scanner/local/scan.go:236-254
//   * filterSecrets (severity part)         pkg/result/filter.go:154-169
//   * JSONWriter                            pkg/report/json.go:22-50 (json.MarshalIndent(report, "", "  ") + "\n")
//   * image-config analyzer input           pkg/fanal/analyzer/imgconf/secret/secret.go:39-62
//                                           (json.MarshalIndent(v1.ConfigFile, "  ", ""))
//   * base-layer secret skip                pkg/fanal/artifact/image/image.go:331-335, 526-554,
//                                           pkg/fanal/image/image.go:111-137
// Go's encoding/json rules are restated where they matter: field order and
// omitempty of the reference's structs (and of go-containerregistry v0.20.3's
// v1.ConfigFile, a dependency absent from the reference tree), HTML-escaped
// strings, json.Indent layout, map keys sorted, time.Time as RFC 3339.
#pragma once
#include <string>
#include <vector>

#include "json.h"
#include "scanner.h"

namespace tsg {

struct LayerRef {                       // ftypes.Layer (pkg/fanal/types/artifact.go:75-79)
  std::string digest, diff_id, created_by;
};

struct ReportOptions {
  long long schema_version = 2;         // report.SchemaVersion (pkg/report/writer.go:24)
  std::string created_at = "0001-01-01T00:00:00Z";   // CreatedAt, RFC 3339 (re-encoded as time.Time marshals)
  std::string artifact_name, artifact_type;
  const JValue* metadata = nullptr;     // types.Metadata as decoded JSON; nullptr = zero Metadata
  std::vector<std::string> severities = {"UNKNOWN", "LOW", "MEDIUM", "HIGH", "CRITICAL"};
  bool layers_sorted = false;           // layers are cached BlobInfo secrets (AnalysisResult.Sort already applied)
};

// The JSON report for the secret results of one artifact: layers[i] are the
// secrets analysed in layer i (lowest first; an fs scan is one layer with an
// empty LayerRef), image_config the image-config analyzer's result (or null).
bool report_json(const std::vector<const SecretVec*>& layers, const std::vector<LayerRef>& refs,
                 const Secret* image_config, const ReportOptions& opt, std::string* out, std::string* err);

// json.Indent(dst, compact, prefix, indent) (encoding/json/indent.go).
void go_indent(const std::string& compact, const std::string& prefix, const std::string& indent, std::string* out);

// json.MarshalIndent(config, "  ", "") of the v1.ConfigFile decoded from
// `config_json` (the image's config blob): the content the image-config
// analyzer scans as "config.json".
bool image_config_content(const std::string& config_json, std::string* out, std::string* err);

// guessBaseLayers: the diff IDs of the layers that belong to the base image
// (their secrets are not scanned), from the image config's history.
bool guess_base_layers(const std::string& config_json, const std::vector<std::string>& diff_ids,
                       std::vector<std::string>* base, std::string* err);

// time.Time JSON round trip: parse an RFC 3339 timestamp (as
// time.Time.UnmarshalJSON accepts it) and format it as MarshalJSON does
// (RFC3339Nano: trailing zeros of the fraction dropped, "Z" for offset 0).
bool go_time_rfc3339(const std::string& in, std::string* out);

}  // namespace tsg
