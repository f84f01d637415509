"""Training-step plumbing for the CLSKD student (config C3): flat parameter / gradient buffers,
Adam as one HIP kernel over the flat buffer, and the batch-sharded gradient all-reduce.

Reference: ``KnowledgeDistillation.configure_optimizers`` returns
``optim.Adam(self.student.parameters(), lr=cfg.learning_rate)`` (distill.py:202-204) and
Lightning's automatic optimisation runs ``loss.backward(); opt.step(); opt.zero_grad()`` per
step.  With ``FlatParams`` the student's parameters live in ONE fp32 buffer (each nn.Parameter a
view), gradients in a second one, so the all-reduce is a single RCCL call (~926 KB) and the
optimizer a single launch.
"""
import torch
import torch.distributed as dist

from . import ops


class FlatParams:
    """Re-homes the trainable parameters of `module` into one contiguous fp32 buffer (their
    .data become views) and keeps a matching gradient buffer."""

    def __init__(self, module):
        self.params = [p for p in module.parameters() if p.requires_grad]
        if not self.params:
            raise ValueError("FlatParams: no trainable parameters")
        dev = self.params[0].device
        # every parameter starts on a 256-B boundary (vector loads of views stay aligned)
        offs, n = [], 0
        for p in self.params:
            offs.append(n)
            n += -(-p.numel() // 64) * 64
        self.data = torch.zeros(n, dtype=torch.float32, device=dev)
        self.grad = torch.zeros(n, dtype=torch.float32, device=dev)
        self.gviews = {}
        with torch.no_grad():
            for p, off in zip(self.params, offs):
                k = p.numel()
                self.data[off:off + k].copy_(p.detach().reshape(-1).float())
                p.data = self.data[off:off + k].view(p.shape)
                self.gviews[p] = self.grad[off:off + k].view(p.shape)
        self.numel = n

    def grad_dict(self):
        return dict(self.gviews)

    def attach_grads(self):
        """Expose the flat gradient as each parameter's .grad (views)."""
        for p in self.params:
            p.grad = self.gviews[p]

    def bump_versions(self):
        """Parameters were rewritten by a kernel: advance their autograd version counters so
        weight-pack caches keyed on (pointer, version) rebuild."""
        torch.autograd.graph.increment_version(self.params)


class FlatAdam:
    """torch.optim.Adam semantics over a FlatParams buffer, one clskd_adam_step launch.

    device_step=True keeps the step count in device memory (`self.t`, int32) and advances it
    in-stream (clskd_adam_step_dev), so a captured training step (clskd.graph.TrainStepGraph)
    replays with the right bias corrections; `step_count` then reads it back."""

    def __init__(self, flat, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0,
                 device_step=False):
        self.flat = flat
        self.lr, self.betas, self.eps, self.weight_decay = lr, betas, eps, weight_decay
        self.m = torch.zeros_like(flat.data)
        self.v = torch.zeros_like(flat.data)
        self.device_step = device_step
        self.t = torch.zeros(1, dtype=torch.int32, device=flat.data.device) if device_step else None
        self._host_steps = 0

    @property
    def step_count(self):
        return int(self.t.item()) if self.device_step else self._host_steps

    def step(self, grad_scale=1.0):
        if self.device_step:
            ops.adam_step_dev(self.flat.data, self.flat.grad, self.m, self.v, self.lr,
                              self.betas[0], self.betas[1], self.eps, self.weight_decay, self.t,
                              grad_scale)
        else:
            self._host_steps += 1
            ops.adam_step(self.flat.data, self.flat.grad, self.m, self.v, self.lr, self.betas[0],
                          self.betas[1], self.eps, self.weight_decay, self._host_steps, grad_scale)
        self.flat.bump_versions()

    def state(self):
        """The optimizer's and the parameters' device state (snapshot / restore)."""
        return [self.flat.data, self.m, self.v] + ([self.t] if self.device_step else [])

    def zero_grad(self):
        ops.fill(self.flat.grad, 0.0)


def allreduce_grads(flat):
    """Sum the flat student gradient across ranks (one RCCL all-reduce over xGMI on GPUs, gloo on
    CPU).  Returns the scale that turns the sum into the mean (passed to FlatAdam.step)."""
    if dist.is_initialized() and dist.get_world_size() > 1:
        dist.all_reduce(flat.grad, op=dist.ReduceOp.SUM)
        return 1.0 / dist.get_world_size()
    return 1.0
