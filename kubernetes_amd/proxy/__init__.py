"""kube-proxy: Service -> Endpoints load balancing on every node.

  config.py     service / endpoints change tracking over shared informers
                (`pkg/proxy/config/config.go`, `pkg/proxy/service.go`, `endpoints.go`)
  iptables.py   iptables proxier: KUBE-SERVICES / KUBE-SVC-* / KUBE-SEP-* / KUBE-XLB-* /
                KUBE-FW-* / KUBE-NODEPORTS chains as one iptables-restore transaction
                (`pkg/proxy/iptables/proxier.go`)
  ipvs.py       IPVS proxier: virtual servers on a dummy interface + real servers
                (`pkg/proxy/ipvs/proxier.go`)
  userspace.py  userspace proxier: an in-process TCP/UDP load balancer per service port with
                round-robin and ClientIP session affinity (`pkg/proxy/userspace/proxier.go`,
                `roundrobin.go`) — the mode that carries real traffic in this environment
  healthcheck.py kube-proxy /healthz and per-service health-check node ports for
                `externalTrafficPolicy: Local` (`pkg/proxy/healthcheck`)
  server.py     ProxyServer wiring (`cmd/kube-proxy/app/server.go:424`)
"""
