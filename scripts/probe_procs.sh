# diagnose per-process GPU memory sources on the GPU box (per-pod VRAM attribution)
set -x
./kubernetes_amd/native/bin/hip-vector-add --hold-mib 1024 --hold-seconds 15 > /tmp/hold.log 2>&1 &
HP=$!
sleep 5
cat /tmp/hold.log
ls -la /proc/$HP/fd | grep -E "dri|kfd"
for f in /proc/$HP/fd/*; do t=$(readlink $f); case "$t" in /dev/dri/*|/dev/kfd) echo "== $f -> $t"; cat /proc/$HP/fdinfo/$(basename $f);; esac; done
cat /proc/$HP/status | grep -i pid
wait $HP
