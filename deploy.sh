#!/usr/bin/env bash
# deploy | redeploy | uninstall — same verbs as the reference's deploy.sh.
# deploy also creates the TLS Secret (gpu-mounter-tls) once, with openssl: a private CA, one
# master⇄worker mTLS certificate per identity (SAN gpu-mounter-worker / gpu-mounter-master) and
# the master API's HTTPS certificate (SAN gpu-mounter-service…, localhost, 127.0.0.1).
set -euo pipefail
cd "$(dirname "$0")"
FILES=(deploy/namespace.yaml deploy/rbac.yaml deploy/placeholder-priority.yaml
       deploy/gpu-mounter-workers.yaml deploy/gpu-mounter-master.yaml deploy/gpu-mounter-svc.yaml
       deploy/networkpolicy.yaml)
NS=kube-system
SECRET=gpu-mounter-tls

pki() {
  kubectl -n "$NS" get secret "$SECRET" >/dev/null 2>&1 && return 0
  local d
  d=$(mktemp -d)
  trap 'rm -rf "$d"' RETURN
  openssl req -x509 -newkey rsa:3072 -nodes -keyout "$d/ca.key" -out "$d/ca.crt" -days 825 \
      -subj "/CN=gpumounter-ca" 2>/dev/null
  for id in worker master; do
    printf 'subjectAltName=DNS:gpu-mounter-%s\nextendedKeyUsage=serverAuth,clientAuth\n' "$id" \
        > "$d/$id.ext"
    openssl req -newkey rsa:3072 -nodes -keyout "$d/$id.key" -out "$d/$id.csr" \
        -subj "/CN=gpu-mounter-$id" 2>/dev/null
    openssl x509 -req -in "$d/$id.csr" -CA "$d/ca.crt" -CAkey "$d/ca.key" -CAcreateserial \
        -out "$d/$id.crt" -days 825 -extfile "$d/$id.ext" 2>/dev/null
  done
  # the master's HTTPS API: the Service's names, and localhost for kubectl port-forward
  local svc=gpu-mounter-service
  printf 'subjectAltName=DNS:%s,DNS:%s.%s,DNS:%s.%s.svc,DNS:%s.%s.svc.cluster.local,DNS:localhost,IP:127.0.0.1\nextendedKeyUsage=serverAuth\n' \
      "$svc" "$svc" "$NS" "$svc" "$NS" "$svc" "$NS" > "$d/master-https.ext"
  openssl req -newkey rsa:3072 -nodes -keyout "$d/master-https.key" -out "$d/master-https.csr" \
      -subj "/CN=$svc" 2>/dev/null
  openssl x509 -req -in "$d/master-https.csr" -CA "$d/ca.crt" -CAkey "$d/ca.key" \
      -CAcreateserial -out "$d/master-https.crt" -days 825 -extfile "$d/master-https.ext" \
      2>/dev/null
  kubectl -n "$NS" create secret generic "$SECRET" --from-file=ca.crt="$d/ca.crt" \
      --from-file=worker.crt="$d/worker.crt" --from-file=worker.key="$d/worker.key" \
      --from-file=master.crt="$d/master.crt" --from-file=master.key="$d/master.key" \
      --from-file=master-https.crt="$d/master-https.crt" \
      --from-file=master-https.key="$d/master-https.key"
}
apply()  { pki; for f in "${FILES[@]}"; do kubectl apply -f "$f"; done; }
remove() {
  for ((i=${#FILES[@]}-1; i>=0; i--)); do kubectl delete --ignore-not-found -f "${FILES[$i]}"; done
  kubectl -n "$NS" delete secret --ignore-not-found "$SECRET"
}
case "${1:-}" in
  deploy) apply ;;
  redeploy) remove; apply ;;
  uninstall) remove ;;
  *) echo "usage: $0 deploy|redeploy|uninstall" >&2; exit 2 ;;
esac
