"""kubeadm: cluster bootstrap for an MI355X node (init / join / token / reset).

Parity: `cmd/kubeadm/app` — phases `certs` (`phases/certs/certs.go:37-260`), `kubeconfig`,
`controlplane` + `etcd` static pod manifests (`phases/controlplane/manifests.go`, default
admission list including ResourceV2 `:45-47`), `uploadconfig`, `markmaster`, bootstrap tokens
(`phases/bootstraptoken/{node,clusterinfo}`), addons (kube-proxy), and `kubeadm join`
token discovery (`discovery/token/token.go`: fetch `kube-public/cluster-info`, verify the JWS made
by the bootstrap signer, pin the CA by `sha256:<SubjectPublicKeyInfo hash>`) followed by the
kubelet's TLS bootstrap.
"""
