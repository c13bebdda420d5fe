"""oracle/ -- TEST INFRASTRUCTURE ONLY.

CPU restatement of the reference render path (oracle.c -> liboracle.so) and
a harness around the unmodified reference sources (ref_harness.c ->
_ref/libref_<W>x<H>.so, buildable only where /root/reference exists).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
import this package, and only as the checker / the timed CPU baseline. The
product package never imports it.
"""
