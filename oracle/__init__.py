# TEST INFRASTRUCTURE -- the CPU oracle (parity checker / CPU baseline).
# Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this.
