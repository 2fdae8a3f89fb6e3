"""TEST INFRASTRUCTURE ONLY — CPU restatement of FederatedScope's aggregators.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s
``cpu_baseline`` leg may import this package, and only as the checker / the
timed CPU baseline.  The product (``federatedscope_amd``) never imports it and
fails loudly when its HIP library is missing.

Parity pin: every function here is checked against golden vectors produced by
the real reference (``tools/gen_golden.py`` → ``tests/golden/*.npz``, see
``tests/test_oracle_golden.py``).
"""
from .fsagg_oracle import *  # noqa: F401,F403
