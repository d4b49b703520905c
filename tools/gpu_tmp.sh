timeout -k 10 200 python tools/uprof.py
