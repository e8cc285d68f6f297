"""rpst — MI355X-native runtime for the RP-Style-Transfer forward path.

`rpst._lib` binds librpst.so (include/rpst.h), `rpst.ops` wraps it for torch device
tensors, `rpst.plan` compiles the reference's nn.Sequential conv stacks into fused conv
launches, `rpst.shard` splits a batch over GPUs and `rpst.synth` makes deterministic
synthetic weights and images.
"""
__all__ = ["ops", "plan", "synth"]
