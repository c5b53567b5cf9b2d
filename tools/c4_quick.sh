set -e
cd /root/repo
timeout -k 10 120 python -u tools/c2_probe.py 0 0
timeout -k 10 200 python -u tools/c4_probe.py 0 4096 3,1
