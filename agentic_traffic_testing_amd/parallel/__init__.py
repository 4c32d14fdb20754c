"""Multi-GPU serving: tensor parallelism (one process per GPU, RCCL over xGMI) and
data-parallel engine replicas behind a router.

* ``comm``             - TP collectives (all-reduce, vocab-parallel sampling, gathers)
* ``tp_engine``        - rank-0 serving engine + TP worker ranks fed by a shm channel
* ``custom_allreduce`` - one-shot IPC all-reduce kernel for small decode messages
* ``dp_router``        - HTTP router over N single-GPU backends (data parallelism)
"""
