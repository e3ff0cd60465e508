// SubjectAccessReview model (see sar.cpp for the reference functions restated).
#pragma once
#include <string>
#include <utility>
#include <vector>

#include "engine.h"

namespace cg {

enum AuthzDecision { AUTHZ_DENY = 0, AUTHZ_ALLOW = 1, AUTHZ_NO_OPINION = 2 };  // k8s authorizer.Decision

struct LabelReq { std::string key, op; std::vector<std::string> values; };
struct FieldReq { std::string field, op, value; };

// authorizer.AttributesRecord subset used by the webhook.
struct Attributes {
  std::string user_name, uid;
  std::vector<std::string> groups;
  std::vector<std::pair<std::string, std::vector<std::string>>> extra;
  std::string verb, ns, api_group, api_version, resource, subresource, name, path;
  bool resource_request = false;
  std::vector<LabelReq> label_sel;
  std::vector<FieldReq> field_sel;
  bool is_read_only() const;
};

Attributes attributes_from_sar(const JVal& sar);
// Returns AUTHZ_* when the request is decided without evaluation (self-allow, system: bypass), else -1.
int authorize_fast_path(const Attributes& a, std::string& reason);
std::string resource_request_to_path(const Attributes& a);
void record_to_cedar(const Attributes& a, std::vector<EntityIn>& ents, RequestIn& req);
// UserToCedarEntity (internal/server/entities/user.go:35-100): group entities, then the principal
void user_to_cedar(const std::string& name, const std::string& uid, const std::vector<std::string>& groups,
                   const std::vector<std::pair<std::string, std::vector<std::string>>>& extra, std::vector<EntityIn>& ents,
                   std::pair<std::string, std::string>& principal);

}  // namespace cg
