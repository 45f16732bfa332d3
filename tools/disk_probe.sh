set -o pipefail
mkdir -p gpurun_out/r03/disk
O=gpurun_out/r03/disk/probe.txt
{ df -hT /var/tmp /tmp . ; cat /proc/mounts | grep -E " / | /var/tmp | /tmp " ; lsblk -o NAME,SIZE,TYPE,MOUNTPOINT,ROTA,MODEL 2>&1 | head -30; } > $O 2>&1
F=/var/tmp/vx_disk_probe.bin
timeout -k 5 120 dd if=/dev/urandom of=$F bs=4M count=768 status=none && sync
python3 - >> $O 2>&1 <<'PY'
import os, time, mmap
F="/var/tmp/vx_disk_probe.bin"
size=os.path.getsize(F)
def drop():
    fd=os.open(F,os.O_RDONLY); os.fsync(fd); os.posix_fadvise(fd,0,0,os.POSIX_FADV_DONTNEED); os.close(fd)
from concurrent.futures import ThreadPoolExecutor
def run(direct, bs, threads):
    drop()
    flags=os.O_RDONLY|(os.O_DIRECT if direct else 0)
    fd=os.open(F,flags)
    n=size//bs
    def work(t):
        buf=mmap.mmap(-1,bs)
        got=0
        for i in range(t,n,threads):
            got+=os.preadv(fd,[buf],i*bs)
        return got
    t0=time.perf_counter()
    with ThreadPoolExecutor(threads) as ex: tot=sum(ex.map(work,range(threads)))
    el=time.perf_counter()-t0
    os.close(fd)
    return tot/el/2**30
for direct in (False, True):
    for bs in (262144, 2097152, 4194304):
        for th in (16,):
            r=[round(run(direct,bs,th),2) for _ in range(2)]
            print(f"direct={direct} bs={bs} threads={th}: {r} GiB/s", flush=True)
PY
rm -f $F
cat $O
