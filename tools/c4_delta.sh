set -e
cd /root/repo
SHD_SSSP_STATS=1 timeout -k 10 120 python -u tools/c4_probe.py 0 4096 3,1
for d in 500000 2000000 5000000 10000000; do SHD_SSSP_STATS=1 SHD_SSSP_DELTA=$d timeout -k 10 120 python -u tools/c4_probe.py 0 4096 3; done
