# What amd-smi / rocm-smi report from inside the tenant-side view (libgm_tenant_view.so), with
# no GPU node, with kfd only, and with kfd + the GPU's render/card nodes granted. Exploratory.
#   gpurun --timeout 300 -- bash bench/gpu_runs/tenant_smi_probe.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/tenant_smi
mkdir -p $O
timeout -k 10 200 python - > $O/probe.txt 2>&1 <<'PY'
import json, os, subprocess, tempfile
from gpumounter_amd.hw.inventory import Inventory
from gpumounter_amd.ops import tenant
inv = Inventory("")
g = inv.gpus()[0]
kfd = inv.kfd_major
root = tempfile.mkdtemp(); cg = tempfile.mkdtemp()
os.makedirs(root + "/dev/dri")
def run(tag, grants, nodes):
    for f in ("dev/kfd", f"dev/dri/renderD{g.render_minor}", f"dev/dri/card{g.card_minor}"):
        p = os.path.join(root, f)
        if os.path.exists(p): os.unlink(p)
    for rel, ma, mi in nodes:
        open(os.path.join(root, rel), "w").write(f"gm-chr {ma}:{mi}\n")
    json.dump({"set": [[2, a, b, 6] for a, b in grants]}, open(cg + "/gm.bpf.json", "w"))
    env = tenant.tenant_env(root, cg)
    for cmd in (["amd-smi", "list", "--json"], ["rocm-smi", "--showuniqueid"]):
        try:
            r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=60)
            print(f"== {tag}: {' '.join(cmd)} rc={r.returncode}\n{r.stdout[-1500:]}\n{r.stderr[-800:]}", flush=True)
        except FileNotFoundError as e:
            print(f"== {tag}: {cmd[0]} missing: {e}")
    print(f"== {tag}: HIP", tenant.hip_devices(root, cg), flush=True)
run("none", [], [])
run("kfd-only", [(kfd, 0)], [("dev/kfd", kfd, 0)])
run("attached", [(kfd, 0), (226, g.render_minor), (226, g.card_minor)],
    [("dev/kfd", kfd, 0), (f"dev/dri/renderD{g.render_minor}", 226, g.render_minor),
     (f"dev/dri/card{g.card_minor}", 226, g.card_minor)])
PY
cat $O/probe.txt | head -150
