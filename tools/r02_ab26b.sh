set -u
for v in os256 base os256 os512; do echo "lib=$v"; LSB_LIBRARY=abtest/$v/liblsb.so timeout -k 10 60 python tools/digit_probe.py 24 2>&1 | tail -2; done
