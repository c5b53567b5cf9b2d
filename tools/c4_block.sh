cd /root/repo
SHD_SSSP_BLOCK=1024 SHD_SSSP_SLOTS=1 timeout -k 10 200 python -u tools/c4_probe.py 0 4096 3 && \
SHD_SSSP_BLOCK=512 SHD_SSSP_SLOTS=2 timeout -k 10 200 python -u tools/c4_probe.py 0 4096 3
