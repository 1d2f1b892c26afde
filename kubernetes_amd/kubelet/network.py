"""Pod networking for the kubelet: network plugins (CNI, kubenet), host-local IPAM, DNS
configuration and host ports.

Parity:
  * `pkg/kubelet/network/plugins.go` (`NetworkPlugin`: Init / SetUpPod / TearDownPod /
    GetPodNetworkStatus / Status, `Event(NET_PLUGIN_EVENT_POD_CIDR_CHANGE)`);
  * `pkg/kubelet/network/cni/cni.go` (first config in `--cni-conf-dir` by name, `.conf` or
    `.conflist`; plugins exec'd from `--cni-bin-dir` with `CNI_COMMAND/CNI_CONTAINERID/CNI_NETNS/
    CNI_IFNAME/CNI_PATH/CNI_ARGS` and the network config on stdin; chained plugins get
    `prevResult`; DEL runs in reverse order);
  * `pkg/kubelet/network/kubenet/kubenet_linux.go` (bridge `cbr0` + host-local IPAM over the
    node's `spec.podCIDR`, status error until the CIDR is known) — host-local here is
    `HostLocalIPAM`, the same on-disk layout as the CNI host-local plugin (one file per reserved
    IP holding the container id, `last_reserved_ip`);
  * `pkg/kubelet/network/dns/dns.go` (`ClusterFirst` / `ClusterFirstWithHostNet` / `Default` /
    `None`+`dnsConfig`, search path `<ns>.svc.<domain> svc.<domain> <domain>` + host searches,
    `ndots:5`, at most 3 nameservers / 6 search domains / 256 characters) and the kubelet-managed
    `/etc/hosts` (`kubelet_pods.go` `makeHostsMount`, hostAliases);
  * `pkg/kubelet/network/hostport/hostport_manager.go` (`KUBE-HOSTPORTS` → `KUBE-HP-<hash>` DNAT
    chains; the host port's socket is opened and held so nothing else can take it).

With the in-process runtimes pods share the node's network namespace, so the plugins allocate
and record addresses (and CNI plugins get an empty `CNI_NETNS`); an OCI runtime with its own
namespaces gets the same calls with a real netns path.
"""
from __future__ import annotations

import asyncio
import shutil
import base64
import hashlib
import ipaddress
import json
import logging
import os
import socket

log = logging.getLogger("kubelet.network")

MAX_NS, MAX_SEARCH, MAX_SEARCH_CHARS = 3, 6, 256


class NetworkError(Exception):
    pass


# ------------------------------------------------------------------------------------ IPAM
class HostLocalIPAM:
    def __init__(self, data_dir, cidr=None):
        self.dir = data_dir
        self.net = None
        if cidr:
            self.set_cidr(cidr)

    def set_cidr(self, cidr):
        self.net = ipaddress.ip_network(cidr, strict=False)
        os.makedirs(self.dir, exist_ok=True)

    @property
    def gateway(self):
        return str(self.net.network_address + 1) if self.net else None

    def _reserved(self):
        out = {}
        for fn in os.listdir(self.dir) if os.path.isdir(self.dir) else ():
            if fn == "last_reserved_ip":
                continue
            try:
                ipaddress.ip_address(fn)
            except ValueError:
                continue
            with open(os.path.join(self.dir, fn)) as f:
                out[fn] = f.read().strip()
        return out

    def allocate(self, container_id):
        if self.net is None:
            raise NetworkError("no pod CIDR configured")
        used = self._reserved()
        for ip, cid in used.items():
            if cid == container_id:
                return ip
        hosts = self.net.num_addresses - 2
        start = 2
        try:
            with open(os.path.join(self.dir, "last_reserved_ip")) as f:
                last = ipaddress.ip_address(f.read().strip())
            if last in self.net:
                start = int(last) - int(self.net.network_address) + 1
        except (OSError, ValueError):
            pass
        for i in range(hosts):
            off = 2 + ((start - 2 + i) % (hosts - 1))
            ip = str(self.net.network_address + off)
            if ip in used:
                continue
            try:
                fd = os.open(os.path.join(self.dir, ip), os.O_WRONLY | os.O_CREAT | os.O_EXCL, 0o644)
            except FileExistsError:
                continue
            with os.fdopen(fd, "w") as f:
                f.write(container_id)
            with open(os.path.join(self.dir, "last_reserved_ip"), "w") as f:
                f.write(ip)
            return ip
        raise NetworkError(f"no IP addresses available in range set: {self.net}")

    def release(self, container_id):
        for ip, cid in self._reserved().items():
            if cid == container_id:
                os.unlink(os.path.join(self.dir, ip))


# ------------------------------------------------------------------------------------ plugins
class NetworkPlugin:
    name = "noop"

    def set_pod_cidr(self, cidr):
        pass

    def status(self):
        return None

    async def setup_pod(self, pod, sandbox_id, netns=""):
        return None

    async def teardown_pod(self, pod, sandbox_id, netns=""):
        pass


class KubenetPlugin(NetworkPlugin):
    """kubenet (`pkg/kubelet/network/kubenet/kubenet_linux.go`): a Linux bridge (`cbr0`) over the
    node's pod CIDR. With a network namespace and the CNI `bridge` / `host-local` / `loopback`
    binaries in `--cni-bin-dir` it delegates exactly as the reference does — the generated
    bridge config (isGateway, ipMasq off, hairpinMode, host-local IPAM over the pod CIDR, the
    bridge MTU) and a loopback ADD — and `--hairpin-mode=promiscuous-bridge` puts the bridge in
    promiscuous mode. Without a namespace (the process runtime shares the host network) it
    allocates from the same host-local range in process."""
    name = "kubenet"

    def __init__(self, data_dir, bridge="cbr0", mtu=1460, cni_bin_dirs=(), hairpin_mode="promiscuous-bridge",
                 non_masquerade_cidr="10.0.0.0/8"):
        self.ipam = HostLocalIPAM(os.path.join(data_dir, "networks", "kubenet"))
        self.bridge, self.mtu = bridge, mtu
        self.cidr = None
        self.bin_dirs = [d for d in cni_bin_dirs if d]
        if hairpin_mode not in ("promiscuous-bridge", "hairpin-veth", "none"):
            raise ValueError(f"invalid hairpin mode {hairpin_mode!r}")
        self.hairpin_mode = hairpin_mode
        self.non_masquerade_cidr = non_masquerade_cidr
        self._promisc_done = False
        self._delegate = None

    def set_pod_cidr(self, cidr):
        if cidr and cidr != self.cidr:
            self.cidr = cidr
            self.ipam.set_cidr(cidr)
            self._delegate = None
            log.info("kubenet: pod CIDR %s, bridge %s gateway %s", cidr, self.bridge, self.ipam.gateway)

    def net_config(self):
        """The bridge network kubenet hands to CNI (NET_CONFIG_TEMPLATE)."""
        return {"cniVersion": "0.1.0", "name": "kubenet", "plugins": [
            {"type": "bridge", "bridge": self.bridge, "mtu": self.mtu, "addIf": "eth0", "isGateway": True,
             "ipMasq": False, "hairpinMode": self.hairpin_mode == "hairpin-veth",
             "ipam": {"type": "host-local", "subnet": self.cidr, "gateway": self.ipam.gateway,
                      "routes": [{"dst": "0.0.0.0/0"}]}}]}

    def _cni(self):
        if self._delegate is None and self.bin_dirs and self.cidr:
            c = CNIPlugin.__new__(CNIPlugin)
            c.conf_dir, c.bin_dirs, c.pod_cidr = None, list(self.bin_dirs), self.cidr
            c.net = self.net_config()
            c._load = lambda: None
            try:
                for typ in ("bridge", "host-local", "loopback"):
                    c._find(typ)
            except NetworkError:
                return None
            self._delegate = c
        return self._delegate

    def status(self):
        if self.cidr is None:
            return "Kubenet does not have netConfig. This is most likely due to lack of PodCIDR"
        return None

    async def _promiscuous(self):
        # PromiscuousBridge: the bridge sees its own pods' hairpin traffic
        if self._promisc_done or self.hairpin_mode != "promiscuous-bridge":
            return
        self._promisc_done = True
        ip = shutil.which("ip")
        if ip:
            p = await asyncio.create_subprocess_exec(ip, "link", "set", self.bridge, "promisc", "on",
                                                     stdout=asyncio.subprocess.DEVNULL, stderr=asyncio.subprocess.DEVNULL)
            await p.wait()

    async def setup_pod(self, pod, sandbox_id, netns=""):
        if self.cidr is None:
            raise NetworkError(self.status())
        cni = self._cni() if netns else None
        if cni is None:
            return self.ipam.allocate(sandbox_id)
        res = await cni._exec("ADD", cni.net["plugins"][0], pod, sandbox_id, netns)
        await cni._exec("ADD", {"type": "loopback"}, pod, sandbox_id, netns)
        await self._promiscuous()
        return result_ip(res)

    async def teardown_pod(self, pod, sandbox_id, netns=""):
        cni = self._cni() if netns else None
        if cni is None:
            self.ipam.release(sandbox_id)
            return
        try:
            await cni._exec("DEL", cni.net["plugins"][0], pod, sandbox_id, netns)
        except NetworkError as e:
            log.warning("%s", e)


class CNIPlugin(NetworkPlugin):
    name = "cni"

    def __init__(self, conf_dir="/etc/cni/net.d", bin_dirs=("/opt/cni/bin",), pod_cidr=None):
        self.conf_dir = conf_dir
        self.bin_dirs = list(bin_dirs)
        self.pod_cidr = pod_cidr
        self.net = None
        self._load()

    def _load(self):
        if not os.path.isdir(self.conf_dir):
            self.net = None
            return
        for fn in sorted(os.listdir(self.conf_dir)):
            if not fn.endswith((".conf", ".conflist", ".json")):
                continue
            with open(os.path.join(self.conf_dir, fn)) as f:
                try:
                    conf = json.load(f)
                except ValueError:
                    continue
            if "plugins" in conf:
                self.net = {"name": conf.get("name", ""), "cniVersion": conf.get("cniVersion", "0.3.1"),
                            "plugins": conf["plugins"]}
            else:
                self.net = {"name": conf.get("name", ""), "cniVersion": conf.get("cniVersion", "0.2.0"), "plugins": [conf]}
            return

    def set_pod_cidr(self, cidr):
        self.pod_cidr = cidr

    def status(self):
        if self.net is None:
            self._load()
        if self.net is None:
            return "cni config uninitialized"
        return None

    def _find(self, typ):
        for d in self.bin_dirs:
            p = os.path.join(d, typ)
            if os.access(p, os.X_OK):
                return p
        raise NetworkError(f'failed to find plugin "{typ}" in path {self.bin_dirs}')

    async def _exec(self, cmd, plugin_conf, pod, sandbox_id, netns, prev=None):
        conf = dict(plugin_conf, name=self.net["name"], cniVersion=self.net["cniVersion"])
        if prev is not None:
            conf["prevResult"] = prev
        if self.pod_cidr and isinstance(conf.get("ipam"), dict) and conf["ipam"].get("subnet") == "usePodCidr":
            conf["ipam"] = dict(conf["ipam"], subnet=self.pod_cidr)
        md = pod["metadata"]
        env = dict(os.environ, CNI_COMMAND=cmd, CNI_CONTAINERID=sandbox_id, CNI_NETNS=netns or "", CNI_IFNAME="eth0",
                   CNI_PATH=os.pathsep.join(self.bin_dirs),
                   CNI_ARGS=f"IgnoreUnknown=1;K8S_POD_NAMESPACE={md.get('namespace', 'default')};"
                            f"K8S_POD_NAME={md['name']};K8S_POD_INFRA_CONTAINER_ID={sandbox_id}")
        p = await asyncio.create_subprocess_exec(self._find(conf["type"]), stdin=asyncio.subprocess.PIPE,
                                                 stdout=asyncio.subprocess.PIPE, stderr=asyncio.subprocess.PIPE, env=env)
        out, err = await p.communicate(json.dumps(conf).encode())
        if p.returncode != 0:
            try:
                msg = json.loads(out).get("msg", "")
            except ValueError:
                msg = (out or err).decode(errors="replace")
            raise NetworkError(f"CNI {cmd} {conf['type']}: {msg.strip() or 'exit ' + str(p.returncode)}")
        if cmd == "ADD" and out.strip():
            return json.loads(out)
        return prev

    async def setup_pod(self, pod, sandbox_id, netns=""):
        if self.status():
            raise NetworkError(self.status())
        res = None
        for pc in self.net["plugins"]:
            res = await self._exec("ADD", pc, pod, sandbox_id, netns, res)
        return result_ip(res)

    async def teardown_pod(self, pod, sandbox_id, netns=""):
        if self.net is None:
            return
        for pc in reversed(self.net["plugins"]):
            try:
                await self._exec("DEL", pc, pod, sandbox_id, netns)
            except NetworkError as e:
                log.warning("%s", e)


def result_ip(res):
    """IPv4 address from a CNI result (0.3.x `ips[]` or 0.2.0 `ip4.ip`)."""
    if not res:
        return None
    for ip in res.get("ips") or ():
        addr = ip.get("address", "")
        if ip.get("version", "4") == "4" and addr:
            return addr.split("/")[0]
    ip4 = (res.get("ip4") or {}).get("ip")
    return ip4.split("/")[0] if ip4 else None


def new_plugin(name, data_dir, cni_conf_dir="/etc/cni/net.d", cni_bin_dir="/opt/cni/bin", hairpin_mode="promiscuous-bridge",
               mtu=1460):
    if name in (None, "", "noop"):
        return NetworkPlugin()
    if name == "kubenet":
        return KubenetPlugin(data_dir, mtu=mtu or 1460, cni_bin_dirs=cni_bin_dir.split(","), hairpin_mode=hairpin_mode)
    if name == "cni":
        return CNIPlugin(cni_conf_dir, cni_bin_dir.split(","))
    raise ValueError(f"unknown network plugin {name!r}")


# ------------------------------------------------------------------------------------ DNS
def parse_resolv_conf_text(data: str):
    """`parseResolvConf` (pkg/kubelet/network/dns/dns.go): nameserver lines accumulate; the last
    search line and the last options line win; lines starting with '#' are comments."""
    ns, search, opts = [], [], []
    for line in data.split("\n"):
        t = line.strip()
        if t.startswith("#"):
            continue
        f = t.split()
        if not f:
            continue
        if f[0] == "nameserver" and len(f) >= 2:
            ns.append(f[1])
        if f[0] == "search":
            search = f[1:]
        if f[0] == "options":
            opts = f[1:]
    return ns, search, opts


def parse_resolv_conf(path):
    try:
        with open(path) as f:
            return parse_resolv_conf_text(f.read())
    except OSError:
        return [], [], []


def omit_duplicates(items):
    seen, out = set(), []
    for x in items:
        if x not in seen:
            seen.add(x)
            out.append(x)
    return out


def merge_dns_options(existing, options):
    """`mergeDNSOptions`: pod dnsConfig options override same-named existing ones."""
    m = {}
    for op in existing:
        k, sep, v = op.partition(":")
        m[k] = v if sep else ""
    for o in options or ():
        m[o.get("name")] = "" if o.get("value") is None else str(o["value"])
    return [k + (":" + v if v else "") for k, v in m.items()]


POD_DNS_CLUSTER, POD_DNS_HOST, POD_DNS_NONE = "cluster", "host", "none"


def get_pod_dns_type(pod):
    """`getPodDNSType`: returns (type, error); None needs the CustomPodDNS gate; ClusterFirst on
    the host network falls back to the host's resolver."""
    from ..utils.features import DefaultFeatureGate
    spec = pod.get("spec") or {}
    policy = spec.get("dnsPolicy") or "ClusterFirst"        # the API default for objects not defaulted
    if policy == "None":
        if DefaultFeatureGate("CustomPodDNS"):
            return POD_DNS_NONE, None
        return POD_DNS_CLUSTER, f"invalid DNSPolicy={policy}: custom pod DNS is disabled"
    if policy == "ClusterFirstWithHostNet":
        return POD_DNS_CLUSTER, None
    if policy == "ClusterFirst":
        return (POD_DNS_HOST if spec.get("hostNetwork") else POD_DNS_CLUSTER), None
    if policy == "Default":
        return POD_DNS_HOST, None
    return POD_DNS_CLUSTER, f"invalid DNSPolicy={policy}"


ETC_HOSTS_PATH = "/etc/hosts"
_HOSTNAME_MAX = 63


def truncate_pod_hostname(pod_name, hostname):
    """`truncatePodHostnameIfNeeded`: at most 63 characters, never ending in '-' or '.'."""
    if len(hostname) <= _HOSTNAME_MAX:
        return hostname
    t = hostname[:_HOSTNAME_MAX].rstrip("-.")
    if not t:
        raise ValueError(f'hostname for pod "{pod_name}" was invalid: "{hostname}"')
    log.error('hostname for pod:"%s" was longer than %d. Truncated hostname to :"%s"', pod_name, _HOSTNAME_MAX, t)
    return t


def generate_pod_hostname_and_domain(pod, cluster_domain):
    """`GeneratePodHostNameAndDomain` (kubelet_pods.go:418): spec.hostname (a DNS label) or the
    pod name, truncated; the domain `<subdomain>.<namespace>.svc.<cluster domain>` with a
    subdomain."""
    from ..api.validation import is_dns1123_label
    md, spec = pod.get("metadata") or {}, pod.get("spec") or {}
    hostname = md.get("name", "")
    if spec.get("hostname"):
        if not is_dns1123_label(spec["hostname"]):
            raise ValueError(f'Pod Hostname "{spec["hostname"]}" is not a valid DNS label')
        hostname = spec["hostname"]
    hostname = truncate_pod_hostname(md.get("name", ""), hostname)
    domain = ""
    if spec.get("subdomain"):
        if not is_dns1123_label(spec["subdomain"]):
            raise ValueError(f'Pod Subdomain "{spec["subdomain"]}" is not a valid DNS label')
        domain = f"{spec['subdomain']}.{md.get('namespace', '')}.svc.{cluster_domain}"
    return hostname, domain


def host_aliases_entries(aliases):
    """`hostsEntriesFromHostAliases`: one "<ip>\t<hostname>" line per hostname."""
    if not aliases:
        return ""
    out = ["", "# Entries added by HostAliases."]
    for a in aliases:
        for h in a.get("hostnames") or ():
            out.append(f"{a.get('ip')}\t{h}")
    return "\n".join(out) + "\n"


def managed_hosts_file_content(ip, hostname, domain, aliases):
    """`managedHostsFileContent`."""
    lines = ["# Kubernetes-managed hosts file.", "127.0.0.1\tlocalhost", "::1\tlocalhost ip6-localhost ip6-loopback",
             "fe00::0\tip6-localnet", "fe00::0\tip6-mcastprefix", "fe00::1\tip6-allnodes", "fe00::2\tip6-allrouters"]
    if domain:
        lines.append(f"{ip}\t{hostname}.{domain}\t{hostname}")
    else:
        lines.append(f"{ip}\t{hostname}")
    return "\n".join(lines) + "\n" + host_aliases_entries(aliases)


def node_hosts_file_content(path, aliases):
    """`nodeHostsFileContent`: the node's hosts file plus the HostAliases entries."""
    try:
        with open(path) as f:
            data = f.read()
    except OSError:
        data = ""
    return data + host_aliases_entries(aliases)


class DNSConfigurer:
    """`pkg/kubelet/network/dns/dns.go` Configurer. `recorder(obj, type, reason, message)` (set
    by the kubelet) receives the DNSConfigForming / MissingClusterDNS / CheckLimitsForResolvConf
    warnings; `node_ref` is the node's object reference."""

    def __init__(self, cluster_dns=(), cluster_domain="cluster.local", resolv_conf="/etc/resolv.conf", node_ip=None,
                 recorder=None, node_ref=None):
        self.cluster_dns = [x for x in cluster_dns if x]
        self.domain = cluster_domain
        self.resolv_conf = resolv_conf
        self.node_ip = node_ip
        self.recorder = recorder
        self.node_ref = node_ref

    def _event(self, obj, reason, msg):
        if self.recorder is not None:
            self.recorder(obj, "Warning", reason, msg)
        else:
            log.warning("%s: %s", reason, msg)

    def form_dns_search_fits_limits(self, search, pod):
        exceeded = False
        if len(search) > MAX_SEARCH:
            search = search[:MAX_SEARCH]
            exceeded = True
        line_len = len(" ".join(search))
        if line_len > MAX_SEARCH_CHARS:
            cut_n = cut_len = 0
            for d in reversed(search):
                cut_len += len(d) + 1
                cut_n += 1
                if line_len - cut_len <= MAX_SEARCH_CHARS:
                    break
            search = search[:len(search) - cut_n]
            exceeded = True
        if exceeded:
            self._event(pod, "DNSConfigForming", "Search Line limits were exceeded, some search paths have been omitted, "
                                                 f"the applied search line is: {' '.join(search)}")
        return search

    def form_dns_nameservers_fits_limits(self, ns, pod):
        if len(ns) > MAX_NS:
            ns = ns[:MAX_NS]
            self._event(pod, "DNSConfigForming", "Nameserver limits were exceeded, some nameservers have been omitted, "
                                                 f"the applied nameserver line is: {' '.join(ns)}")
        return ns

    def _cluster_searches(self, host_search, pod):
        if not self.domain:
            return list(host_search)
        ns = pod["metadata"].get("namespace", "")
        return omit_duplicates([f"{ns}.svc.{self.domain}", f"svc.{self.domain}", self.domain] + list(host_search))

    def check_limits_for_resolv_conf(self):
        """`CheckLimitsForResolvConf`: warn (on the node) when the host's search line leaves no
        room for the cluster domains."""
        try:
            with open(self.resolv_conf) as f:
                _, search, _ = parse_resolv_conf_text(f.read())
        except OSError as e:
            self._event(self.node_ref, "CheckLimitsForResolvConf", str(e))
            return
        limit = MAX_SEARCH - (3 if self.domain else 0)
        if len(search) > limit:
            self._event(self.node_ref, "CheckLimitsForResolvConf",
                        f"Resolv.conf file '{self.resolv_conf}' contains search line consisting of more than {limit} domains!")
        elif len(" ".join(search)) > MAX_SEARCH_CHARS:
            self._event(self.node_ref, "CheckLimitsForResolvConf",
                        f"Resolv.conf file '{self.resolv_conf}' contains search line which length is more than allowed "
                        f"{MAX_SEARCH_CHARS} chars!")

    def pod_dns(self, pod):
        """`GetPodDNS`: (nameservers, searches, options)."""
        from ..utils.features import DefaultFeatureGate
        spec = pod.get("spec") or {}
        if self.resolv_conf:
            ns, search, opts = parse_resolv_conf(self.resolv_conf)
        else:
            ns, search, opts = [], [], []
        typ, err = get_pod_dns_type(pod)
        if err:
            log.warning("failed to get DNS type for pod %s: %s; falling back to ClusterFirst", pod["metadata"].get("name"),
                        err)
        if typ == POD_DNS_NONE:
            ns, search, opts = [], [], []
        elif typ == POD_DNS_CLUSTER and self.cluster_dns:
            ns, search, opts = list(self.cluster_dns), self._cluster_searches(search, pod), ["ndots:5"]
        else:
            if typ == POD_DNS_CLUSTER:
                msg = ('kubelet does not have ClusterDNS IP configured and cannot create Pod using "ClusterFirst" '
                       'policy. Falling back to "Default" policy.')
                self._event(self.node_ref, "MissingClusterDNS", msg)
                md = pod["metadata"]
                self._event(pod, "MissingClusterDNS", f'pod: "{md.get("name")}_{md.get("namespace", "")}'
                                                      f'({md.get("uid", "")})". {msg}')
            if not self.resolv_conf:
                ns = ["::1"] if self.node_ip and ":" in str(self.node_ip) else ["127.0.0.1"]
                search = ["."]
        cfg = spec.get("dnsConfig")
        if cfg is not None and DefaultFeatureGate("CustomPodDNS"):
            ns = omit_duplicates(ns + list(cfg.get("nameservers") or ()))
            search = omit_duplicates(search + list(cfg.get("searches") or ()))
            opts = merge_dns_options(opts, cfg.get("options"))
        return self.form_dns_nameservers_fits_limits(ns, pod), self.form_dns_search_fits_limits(search, pod), opts

    def resolv_text(self, pod):
        ns, search, opts = self.pod_dns(pod)
        lines = [f"nameserver {x}" for x in ns]
        if search:
            lines.append("search " + " ".join(search))
        if opts:
            lines.append("options " + " ".join(opts))
        return "\n".join(lines) + "\n"

    def pod_hostname_and_domain(self, pod):
        """`GeneratePodHostNameAndDomain`."""
        return generate_pod_hostname_and_domain(pod, self.domain)

    def hosts_text(self, pod, ip):
        """`ensureHostsFile`: the kubelet-managed file, or for a host-network pod the node's own
        /etc/hosts; HostAliases appended either way."""
        spec = pod.get("spec") or {}
        if spec.get("hostNetwork"):
            return node_hosts_file_content(ETC_HOSTS_PATH, spec.get("hostAliases"))
        try:
            host, domain = self.pod_hostname_and_domain(pod)
        except ValueError as e:         # validation keeps these out; never fail the sync over it
            log.warning("%s", e)
            host, domain = (pod.get("metadata") or {}).get("name", ""), ""
        return managed_hosts_file_content(ip, host, domain, spec.get("hostAliases"))

    def write_pod_files(self, pod_dir, pod, ip, hosts_only=False):
        """Write `etc-hosts` and `resolv.conf` under the pod dir; returns the container mounts.
        hosts_only: no cluster DNS is configured — the kubelet still manages /etc/hosts of every
        pod (`makeHostsMount`), resolv.conf stays the runtime's."""
        os.makedirs(pod_dir, exist_ok=True)
        mounts = []
        # makeMounts: every pod with an IP gets a kubelet-written /etc/hosts (a host-network pod
        # the node's own plus its HostAliases)
        if ip:
            hp = os.path.join(pod_dir, "etc-hosts")
            with open(hp, "w") as f:
                f.write(self.hosts_text(pod, ip))
            mounts.append({"containerPath": "/etc/hosts", "hostPath": hp, "readOnly": False})
        if hosts_only:
            return mounts
        rp = os.path.join(pod_dir, "resolv.conf")
        with open(rp, "w") as f:
            f.write(self.resolv_text(pod))
        mounts.append({"containerPath": "/etc/resolv.conf", "hostPath": rp, "readOnly": False})
        return mounts


# ------------------------------------------------------------------------------------ hostports
def _chain(name, proto, port):
    h = hashlib.sha256(f"{name}{port}{proto}".encode()).digest()
    return "KUBE-HP-" + base64.b32encode(h).decode()[:16]


def make_port_mappings(container):
    """`kubecontainer.MakePortMappings`: one mapping per container port, named
    `<container>-<name>` or `<container>-<PROTO>:<port>`; a repeated name is dropped (the same
    protocol/port exposed twice)."""
    out, names = [], set()
    for p in container.get("ports") or ():
        proto = p.get("protocol") or "TCP"
        name = (f"{container.get('name', '')}-{p['name']}" if p.get("name")
                else f"{container.get('name', '')}-{proto}:{int(p.get('containerPort') or 0)}")
        if name in names:
            log.warning("Port name conflicted, %r is defined more than once", name)
            continue
        names.add(name)
        out.append({"name": name, "protocol": proto, "containerPort": int(p.get("containerPort") or 0),
                    "hostPort": int(p.get("hostPort") or 0), "hostIP": p.get("hostIP") or ""})
    return out


class HostportManager:
    def __init__(self, hold_sockets=True):
        self.hold = hold_sockets
        self.held: dict[tuple, socket.socket] = {}          # (proto, hostIP, port) -> socket
        self.mappings: dict[str, list] = {}                 # pod uid -> [(proto, hostIP, hostPort, containerPort, podIP, name)]

    @staticmethod
    def pod_mappings(pod, ip):
        out = []
        md = pod["metadata"]
        full = f"{md['name']}_{md.get('namespace', 'default')}"
        for c in (pod.get("spec") or {}).get("containers") or ():
            for pm in make_port_mappings(c):
                if pm["hostPort"]:
                    out.append((pm["protocol"].lower(), pm["hostIP"], pm["hostPort"], pm["containerPort"], ip, full))
        return out

    def add(self, pod, ip):
        if (pod.get("spec") or {}).get("hostNetwork"):
            return []
        maps = self.pod_mappings(pod, ip)
        opened = []
        try:
            for proto, hip, hport, _, _, _ in maps:
                key = (proto, hip, hport)
                if key in self.held or not self.hold:
                    continue
                s = socket.socket(socket.AF_INET, socket.SOCK_STREAM if proto == "tcp" else socket.SOCK_DGRAM)
                try:
                    s.bind((hip or "0.0.0.0", hport))
                    if proto == "tcp":
                        s.listen(1)
                except OSError as e:
                    s.close()
                    raise NetworkError(f'cannot open "{proto}:{hport}" for the pod\'s host port: {e}')
                self.held[key] = s
                opened.append(key)
        except NetworkError:
            for k in opened:
                self.held.pop(k).close()
            raise
        self.mappings[pod["metadata"]["uid"]] = maps
        return maps

    def remove(self, pod):
        maps = self.mappings.pop(pod["metadata"]["uid"], [])
        for proto, hip, hport, _, _, _ in maps:
            s = self.held.pop((proto, hip, hport), None)
            if s is not None:
                s.close()

    def rules(self):
        """`iptables-restore` input for the nat table."""
        lines = ["*nat", ":KUBE-HOSTPORTS - [0:0]"]
        body = []
        for maps in self.mappings.values():
            for proto, hip, hport, cport, ip, name in maps:
                ch = _chain(name, proto, hport)
                lines.append(f":{ch} - [0:0]")
                dst = f" -d {hip}/32" if hip else ""
                body.append(f'-A KUBE-HOSTPORTS -m comment --comment "{name} hostport {hport}" -m {proto} -p {proto}'
                            f"{dst} --dport {hport} -j {ch}")
                body.append(f'-A {ch} -m comment --comment "{name} hostport {hport}" -s {ip}/32 -j KUBE-MARK-MASQ')
                body.append(f'-A {ch} -m comment --comment "{name} hostport {hport}" -m {proto} -p {proto} '
                            f"-j DNAT --to-destination {ip}:{cport}")
        return "\n".join(lines + body + ["COMMIT"]) + "\n"

    def close(self):
        for s in self.held.values():
            s.close()
        self.held.clear()


# ------------------------------------------------------------------------------------ node IP
def host_ip_addresses():
    """The addresses assigned to this host's interfaces (`net.InterfaceAddrs`): IPv4 through
    SIOCGIFADDR on each interface, IPv6 from /proc/net/if_inet6."""
    import fcntl
    import ipaddress
    import struct
    out = set()
    try:
        names = [n for _, n in socket.if_nameindex()]
    except OSError:
        names = []
    s4 = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
    try:
        for n in names:
            try:
                raw = fcntl.ioctl(s4.fileno(), 0x8915, struct.pack("256s", n[:15].encode()))    # SIOCGIFADDR
                out.add(socket.inet_ntoa(raw[20:24]))
            except OSError:
                continue
    finally:
        s4.close()
    try:
        with open("/proc/net/if_inet6") as f:
            for line in f:
                h = line.split()[0]
                out.add(str(ipaddress.IPv6Address(int(h, 16))))
    except OSError:
        pass
    return out


def validate_node_ip(node_ip, host_addrs=None):
    """`validateNodeIP` (kubelet_node_status.go): a valid unicast address that is neither
    loopback, multicast, link-local nor unspecified, and is assigned to this host. Raises
    ValueError with the reference message."""
    import ipaddress
    try:
        ip = ipaddress.ip_address(str(node_ip or "").strip())
    except ValueError:
        raise ValueError("nodeIP must be a valid IP address") from None
    if ip.is_loopback:
        raise ValueError("nodeIP can't be loopback address")
    if ip.is_multicast:
        raise ValueError("nodeIP can't be a multicast address")
    if ip.is_link_local:
        raise ValueError("nodeIP can't be a link-local unicast address")
    if ip.is_unspecified:
        raise ValueError("nodeIP can't be an all zeros address")
    addrs = host_ip_addresses() if host_addrs is None else host_addrs
    if not any(ipaddress.ip_address(a) == ip for a in addrs if a):
        raise ValueError(f'Node IP: "{ip}" not found in the host\'s network interfaces')
