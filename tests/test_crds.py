"""CRD schema parity with the reference manifests (structure, types, enums,
defaults, required, names), ignoring description text."""
import os

import pytest
import yaml

from operator_amd.api import crds
from operator_amd.api.models import AIProvider, PatternLibrary, Podmortem

REF = "/root/reference/src/main/kubernetes"


def _strip(o):
    if isinstance(o, dict):
        return {k: _strip(v) for k, v in o.items() if k != "description"}
    if isinstance(o, list):
        return [_strip(v) for v in o]
    return o


@pytest.mark.parametrize("fname,fn", [("podmortem-crd.yaml", crds.podmortem_crd),
                                      ("patternlibrary-crd.yaml", crds.patternlibrary_crd),
                                      ("aiprovider-crd.yaml", crds.aiprovider_crd)])
def test_crd_matches_reference(fname, fn):
    path = os.path.join(REF, fname)
    if not os.path.exists(path):
        pytest.skip("reference manifests not mounted")
    with open(path) as f:
        ref = yaml.safe_load(f)
    ours = fn()
    assert ours["metadata"] == ref["metadata"]
    assert _strip(ours["spec"]) == _strip(ref["spec"])


def test_render_all_is_valid_yaml():
    docs = list(yaml.safe_load_all(crds.render_all()))
    kinds = [d["kind"] for d in docs]
    assert kinds.count("CustomResourceDefinition") == 3
    assert "ClusterRole" in kinds and "Deployment" in kinds
    role = next(d for d in docs if d["kind"] == "ClusterRole")
    assert any("apps" in r["apiGroups"] for r in role["rules"])  # Q9 fix


def test_models_round_trip_reference_examples():
    pm = Podmortem.model_validate({
        "apiVersion": "podmortem.redhat.com/v1alpha1", "kind": "Podmortem",
        "metadata": {"name": "quarkus-app-monitor"},
        "spec": {"podSelector": {"matchLabels": {"app": "quarkus-app"}}, "aiAnalysisEnabled": True,
                 "aiProviderRef": {"name": "openai-provider", "namespace": "podmortem-system"}}})
    assert pm.spec.ai_provider_ref.namespace == "podmortem-system"
    assert pm.to_obj()["spec"]["podSelector"]["matchLabels"] == {"app": "quarkus-app"}
    pl = PatternLibrary.model_validate({"metadata": {"name": "q"}, "spec": {"repositories": [
        {"name": "core-patterns", "url": "https://example/p.git", "branch": "main"}], "refreshInterval": "1h"}})
    assert pl.spec.repositories[0].branch == "main"
    ap = AIProvider.model_validate({"metadata": {"name": "o"}, "spec": {
        "providerId": "openai", "apiUrl": "https://api.openai.com/v1", "modelId": "gpt-3.5-turbo",
        "authenticationRef": {"secretName": "openai-credentials", "secretKey": "api-key"}, "unknownField": 1}})
    assert ap.spec.authentication_ref.secret_key == "api-key"
    assert ap.to_obj()["spec"]["unknownField"] == 1  # extra fields preserved
