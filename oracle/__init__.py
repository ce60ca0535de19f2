"""CPU oracle for the denoise-gan hot path — test infrastructure only.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
import this package; the product path (denoise-gan_amd/) never does.
"""
