"""MI355X-native A2C/ACKTR engine with the public API of jrobine/actor-critic.

Modules mirror the reference package (reference: actorcritic/__init__.py:1-16):
`agents`, `model`, `envs.atari.model`, `objectives`, `policies`, `baselines`, `nn`,
`kfac_utils`, `multi_env`, `envs.atari.wrappers`; plus `session` (the TF-session
stand-in) and `parallel` (one process per GPU over RCCL).  The arithmetic runs in
libacmi.so (hand-written HIP for gfx950); see DESIGN.md.
"""
