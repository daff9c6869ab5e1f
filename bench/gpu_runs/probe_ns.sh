# What the unprivileged GPU box allows for namespaced tenants (user + mount namespaces, bind
# mounts of the GPU device nodes). No GPU work; every step is bounded.
#   gpurun --timeout 120 -- bash bench/gpu_runs/probe_ns.sh
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/probe_ns
mkdir -p "$O"
{
id; uname -r
cat /proc/sys/user/max_user_namespaces /proc/sys/kernel/unprivileged_userns_clone 2>&1
cat /proc/sys/kernel/apparmor_restrict_unprivileged_userns 2>&1
ls -la /dev/kfd /dev/dri 2>&1
stat -c '%n %d %i %t:%T' /dev /dev/kfd /dev/dri /dev/dri/* 2>&1
grep -E ' /dev| /sys | /proc ' /proc/self/mountinfo
cat /proc/self/status | grep -E 'Cap|Seccomp|NoNewPrivs'
cat /proc/self/cgroup; stat -fc %T /sys/fs/cgroup
echo "--- unshare -Ur"
timeout 10 unshare -Ur id 2>&1; echo rc=$?
echo "--- unshare -Urm bind kfd"
timeout 10 unshare -Urm --propagation private bash -c '
  mkdir -p /tmp/nsd && mount -t tmpfs tmpfs /tmp/nsd && touch /tmp/nsd/kfd &&
  mount --bind /dev/kfd /tmp/nsd/kfd && ls -la /tmp/nsd && exec 3<>/tmp/nsd/kfd && echo open-ok' 2>&1; echo rc=$?
echo "--- unshare -Urmpf"
timeout 10 unshare -Urmpf --mount-proc id 2>&1; echo rc=$?
python3 -c "import os; print(hasattr(os,'unshare'), os.cpu_count())"
} > "$O/probe.txt" 2>&1
cat "$O/probe.txt"
