set -e
cd /root/repo
timeout -k 10 120 python -u tools/c4_probe.py 0 4096 3
for d in 8000000; do SHD_SSSP_DELTA=$d timeout -k 10 120 python -u tools/c4_probe.py 0 4096 3; done
SHD_SSSP_SLOTS=3 timeout -k 10 120 python -u tools/c4_probe.py 0 4096 3
