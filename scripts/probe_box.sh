set -x
id
grep -i cap /proc/self/status
cat /proc/sys/user/max_user_namespaces
cat /proc/sys/kernel/unprivileged_userns_clone 2>&1
unshare -Ur true && echo USERNS_OK
unshare -Urm sh -c 'mount -t tmpfs t /tmp && echo TMPFS_OK'
unshare -Urmpf --mount-proc sh -c 'echo PIDNS_OK; ps -e | head -3'
mount | grep -E 'cgroup|/dev '
cat /proc/self/cgroup
ls -l /dev/kfd /dev/dri
ls /sys/class/kfd/kfd/topology/nodes
cat /sys/fs/cgroup/cgroup.controllers 2>&1
ls -ld /sys/fs/cgroup/$(cut -d: -f3 /proc/self/cgroup | head -1)
nproc; free -g
ls /opt/rocm/lib/libamd_smi* 
