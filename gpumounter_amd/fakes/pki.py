"""Throw-away PKI for hermetic deployments: the master⇄worker mTLS material deploy.sh puts into
the ``gpu-mounter-tls`` Secret, made with the ``openssl`` CLI (ECDSA P-256, 2 days).

The worker's certificate carries ``DNS:gpu-mounter-worker`` (``tls_server_name``) and the
master's ``DNS:gpu-mounter-master`` (the worker's ``tls_client_names``), as in the shipped
manifests; ``master-https`` is the master API's serving certificate (the Service's names and
127.0.0.1); the reference dials the worker without TLS (reference: cmd/GPUMounter-master/
main.go:82,185).
"""
from __future__ import annotations

import os
import subprocess
from typing import Dict


def _openssl(cwd: str, *args: str) -> None:
    subprocess.run(["openssl", *args], cwd=cwd, check=True, capture_output=True, timeout=60)


def make_pki(d: str, names: Dict[str, str] = None) -> Dict[str, str]:
    """CA + one certificate per ``{file stem: DNS SAN}`` in ``d``. Returns the paths:
    ``ca``, and ``<stem>.crt`` / ``<stem>.key`` for every stem."""
    names = names or {"worker": "gpu-mounter-worker", "master": "gpu-mounter-master",
                      # the master's HTTPS API (GM_MASTER_TLS_CERT): the Service names and the
                      # loopback address hermetic clients use
                      "master-https": "DNS:gpu-mounter-service,DNS:gpu-mounter-service."
                                      "kube-system.svc,DNS:localhost,IP:127.0.0.1"}
    os.makedirs(d, exist_ok=True)
    ec = ("-newkey", "ec", "-pkeyopt", "ec_paramgen_curve:prime256v1", "-nodes")
    _openssl(d, "req", "-x509", *ec, "-keyout", "ca.key", "-out", "ca.crt", "-days", "2",
             "-subj", "/CN=gm-hermetic-ca")
    out = {"ca": os.path.join(d, "ca.crt")}
    for stem, dns in names.items():
        # "name" → DNS:name; "DNS:a,IP:127.0.0.1" → that subjectAltName as given (CN: the first)
        san = dns if ":" in dns else f"DNS:{dns}"
        cn = san.split(",")[0].split(":", 1)[1]
        with open(os.path.join(d, f"{stem}.ext"), "w") as fh:
            fh.write(f"subjectAltName={san}\n")
        _openssl(d, "req", *ec, "-keyout", f"{stem}.key", "-out", f"{stem}.csr",
                 "-subj", f"/CN={cn}")
        _openssl(d, "x509", "-req", "-in", f"{stem}.csr", "-CA", "ca.crt", "-CAkey", "ca.key",
                 "-CAcreateserial", "-out", f"{stem}.crt", "-days", "2", "-extfile",
                 f"{stem}.ext")
        out[f"{stem}.crt"] = os.path.join(d, f"{stem}.crt")
        out[f"{stem}.key"] = os.path.join(d, f"{stem}.key")
    return out
