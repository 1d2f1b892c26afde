"""Component configuration: scheduler Policy (file / ConfigMap / providers / validation),
KubeSchedulerConfiguration, KubeProxyConfiguration and AdmissionConfiguration files."""
import argparse

import pytest
import yaml

from kubernetes_amd.scheduler import policy as SP


def test_policy_parse_and_providers(run):
    preds, prios, ext = SP.parse_policy('{"kind":"Policy","predicates":[{"name":"PodFitsResources"},'
                                        '{"name":"CheckVolumeBinding"}],"priorities":[{"name":"MostRequestedPriority",'
                                        '"weight":2}],"extenders":[{"urlPrefix":"http://x","filterVerb":"filter"}]}')
    assert preds == ["PodFitsResources", "CheckVolumeBinding"] and prios == {"MostRequestedPriority": 2}
    assert ext[0]["urlPrefix"] == "http://x"
    for bad in ('{"predicates":[{"name":"Nope"}]}', '{"priorities":[{"name":"LeastRequestedPriority","weight":0}]}',
                '{"kind":"Deployment"}'):
        with pytest.raises(SP.PolicyError):
            SP.parse_policy(bad)

    class CM:
        async def get(self, res, name, ns):
            assert (res, name, ns) == ("configmaps", "sched-policy", "kube-system")
            return {"data": {"policy.cfg": "kind: Policy\npriorities:\n- name: ImageLocalityPriority\n  weight: 3\n"}}

    async def main():
        p, w, _ = await SP.resolve_algorithm(CM(), policy_configmap="sched-policy")
        assert p is None and w == {"ImageLocalityPriority": 3}
        p, w, _ = await SP.resolve_algorithm(None, provider="ClusterAutoscalerProvider")
        assert "MostRequestedPriority" in w and "LeastRequestedPriority" not in w
        with pytest.raises(SP.PolicyError):
            await SP.resolve_algorithm(None, provider="Bogus")
    run(main())


def test_proxy_config_file(tmp_path):
    from kubernetes_amd.cmd.proxy import apply_config_file
    p = tmp_path / "kp.yaml"
    p.write_text(yaml.safe_dump({"apiVersion": "kubeproxy.config.k8s.io/v1alpha1", "kind": "KubeProxyConfiguration",
                                 "mode": "ipvs", "clusterCIDR": "10.244.0.0/16", "ipvs": {"scheduler": "lc"},
                                 "iptables": {"masqueradeAll": True, "syncPeriod": "45s", "minSyncPeriod": "500ms"},
                                 "metricsBindAddress": "0.0.0.0:10249", "healthzBindAddress": "0.0.0.0:10256"}))
    a = argparse.Namespace(proxy_mode="iptables", cluster_cidr="", bind_address="127.0.0.1", hostname_override="h",
                           masquerade_all=False, iptables_sync_period=30.0, iptables_min_sync_period=0.0,
                           ipvs_scheduler="rr", healthz_port=1, metrics_port=2, kubeconfig=None)
    apply_config_file(a, str(p))
    assert (a.proxy_mode, a.cluster_cidr, a.ipvs_scheduler, a.masquerade_all) == ("ipvs", "10.244.0.0/16", "lc", True)
    assert a.iptables_sync_period == 45 and a.iptables_min_sync_period == 0.5 and a.metrics_port == 10249


def test_admission_config_file(tmp_path):
    from kubernetes_amd.cmd.apiserver import load_admission_config
    (tmp_path / "erl.yaml").write_text(yaml.safe_dump({"kind": "Configuration", "limits": [{"type": "Server", "qps": 5,
                                                                                            "burst": 10}]}))
    (tmp_path / "adm.yaml").write_text(yaml.safe_dump({
        "apiVersion": "apiserver.k8s.io/v1alpha1", "kind": "AdmissionConfiguration",
        "plugins": [{"name": "EventRateLimit", "path": "erl.yaml"},
                    {"name": "PodTolerationRestriction", "configuration": {"default": []}}]}))
    cfg = load_admission_config(str(tmp_path / "adm.yaml"))
    assert cfg["EventRateLimit"]["limits"][0]["qps"] == 5 and cfg["PodTolerationRestriction"] == {"default": []}
