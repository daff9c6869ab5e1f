#!/usr/bin/env bash
# deploy | redeploy | uninstall — same verbs as the reference's deploy.sh.
set -euo pipefail
cd "$(dirname "$0")"
FILES=(deploy/namespace.yaml deploy/rbac.yaml deploy/placeholder-priority.yaml
       deploy/gpu-mounter-workers.yaml deploy/gpu-mounter-master.yaml deploy/gpu-mounter-svc.yaml)
apply()  { for f in "${FILES[@]}"; do kubectl apply -f "$f"; done; }
remove() { for ((i=${#FILES[@]}-1; i>=0; i--)); do kubectl delete --ignore-not-found -f "${FILES[$i]}"; done; }
case "${1:-}" in
  deploy) apply ;;
  redeploy) remove; apply ;;
  uninstall) remove ;;
  *) echo "usage: $0 deploy|redeploy|uninstall" >&2; exit 2 ;;
esac
