// Admission webhook model (admission.cpp): AdmissionReview request -> (EntityMap, Request).
#pragma once
#include <string>
#include <utility>
#include <vector>

#include "sar.h"

namespace cg {

// admission.Request fields the reference reads (sigs.k8s.io/controller-runtime admission.Request
// over k8s.io/api/admission/v1 AdmissionRequest)
struct AdmissionRequest {
  std::string uid, operation, name, ns, sub_resource;
  std::string kind_group, kind_version, kind;       // req.Kind
  std::string res_group, res_version, resource;     // req.Resource
  std::string username, user_uid;                   // req.UserInfo
  std::vector<std::string> groups;
  std::vector<std::pair<std::string, std::vector<std::string>>> extra;
  bool has_object = false, has_old = false;         // RawExtension.Raw != nil
  JVal object, old_object;
};

// outcome of admission_to_cedar
enum AdmissionOutcome { ADM_EVAL = 0, ADM_SKIP = 1, ADM_ERROR = 2 };

// An AdmissionReview ({"request": {...}}) or a bare request object.
AdmissionRequest admission_request_from_json(const JVal& review);
// handler.go:43-153 up to IsAuthorized: ADM_SKIP for the skipped namespaces (allowed without
// evaluation), ADM_ERROR with the reference's wrapped error text (admission.Errored, HTTP 500),
// else ADM_EVAL with the entities and request.
int admission_to_cedar(const AdmissionRequest& a, std::vector<EntityIn>& ents, RequestIn& req, std::string& err);

}  // namespace cg
