"""CPU oracle for the SAC gradient-step hot path — TEST INFRASTRUCTURE ONLY.

Nothing under ``oracle/`` is part of the product.  Only ``tests/``,
``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import it,
and only as the checker (or, for the baseline, as the timed CPU port).  The product
path (``humanoid-walking-with-sac_amd/``) never imports it and fails loudly when its
HIP library is missing.

Contents
--------
pyrandom   exact restatement of CPython's MT19937 + ``random.sample`` (uniform
           replay indices, /usr/lib/python3.10/random.py:239-249,406-504) and of
           numpy's legacy ``random_sample`` (PER uniforms).
sac_step   functional torch-CPU restatement of ``SAC.update_parameters``
           (reference ``sac_imp.py:74-152`` + ``networks_model1.py:27-99``), fp32 or
           fp64, with injected minibatch / eps so one step is fully determined.
per        numpy restatement of ``PrioritizedReplayBuffer`` sample / push /
           update_priorities (reference ``replay_buffer.py:25-90``).
replay_ref deque-of-tuples uniform buffer with the reference's data path
           (``replay_buffer.py:5-22``), used only to time the CPU baseline.

Parity pinning: ``tests/golden/*.npz`` were produced by ``tools/make_golden.py``,
which imports the reference from /root/reference in the build container and runs
it.  ``tests/test_oracle.py`` checks this oracle against those fixtures (bit-exact
for indices, bit-exact for the fp32 step on the captured minibatch/eps).
"""
