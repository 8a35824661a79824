"""CPU oracle for the INSR-PDE training-loop hot path — TEST INFRASTRUCTURE ONLY.

This module is the checker, never the product: only ``tests/``,
``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import it.
The shipped path (``insr-pde_amd/base``) runs on the HIP library and fails loudly
without it; nothing in the product imports this file.

It restates, in plain PyTorch fp32 on the CPU, the reference algorithm that the
HIP kernels replace.  Every function cites the reference file:line it follows
(paths relative to the reference root, qingxu-thu/INSR-PDE @ 2025-01-14):

* SIREN field network and its initialisation .... base/networks.py:12-93
* autograd spatial derivatives ................... base/diff_ops.py:6-82
* collocation samplers ........................... base/sampling.py:4-64
* phase residuals ................................ advection/model.py:43-91,
                                                   fluid/model.py:42-151,
                                                   elasticity/model.py:109-189,
                                                   elasticity/losses.py:6-39
* initial conditions ............................. advection/examples.py:14-16,
                                                   fluid/examples.py:17-51
* optimiser + LR schedule ........................ base/baseModel.py:55-62,73-81
                                                   (torch.optim.Adam defaults,
                                                   ReduceLROnPlateau)

Parity pin: ``tests/golden/make_golden.py`` imports the reference itself in the
build container and records its outputs on fixed weights/samples;
``tests/test_oracle_golden.py`` checks this restatement against those vectors.
"""
import math

import torch
import torch.nn as nn

OMEGA = 30.0  # base/networks.py:27 -- sin(30 * input)


# --------------------------------------------------------------------------
# SIREN network (base/networks.py:20-93)
# --------------------------------------------------------------------------
class _SineAct(nn.Module):
    """sin(30 z) (base/networks.py:21-27)."""

    def forward(self, z):
        return torch.sin(OMEGA * z)


class OracleSiren(nn.Module):
    """in -> W -> (L x W->W) -> out, sine after every layer but the last.

    Layer list and init follow base/networks.py:31-65: every nn.Linear is first
    built with torch's default init (weight kaiming-uniform, bias U(+-1/sqrt(fan_in))),
    then every weight is redrawn U(+-sqrt(6/fan_in)/30) (sine_init :80-85) in
    module order, then layer 0's weight is redrawn U(+-1/fan_in)
    (first_layer_sine_init :88-93).  Biases keep the nn.Linear default.
    The RNG stream is consumed in exactly that order, so a given torch seed
    reproduces the reference's weights bit for bit.
    """

    def __init__(self, d_in, d_out, num_hidden_layers, hidden_features):
        super().__init__()
        mods = [nn.Linear(d_in, hidden_features), _SineAct()]
        for _ in range(num_hidden_layers):
            mods += [nn.Linear(hidden_features, hidden_features), _SineAct()]
        mods.append(nn.Linear(hidden_features, d_out))
        self.net = nn.Sequential(*mods)
        with torch.no_grad():
            for m in self.net:
                if isinstance(m, nn.Linear):
                    fan_in = m.weight.shape[1]
                    bound = math.sqrt(6.0 / fan_in) / OMEGA
                    m.weight.uniform_(-bound, bound)
            w0 = self.net[0].weight
            w0.uniform_(-1.0 / w0.shape[1], 1.0 / w0.shape[1])

    def forward(self, coords):
        return self.net(coords)

    def linears(self):
        return [m for m in self.net if isinstance(m, nn.Linear)]


def flat_params(net):
    """All parameters in state_dict order (net.0.weight, net.0.bias, net.2.weight ...)."""
    return torch.cat([p.detach().reshape(-1) for p in net.parameters()])


def flat_grads(net):
    return torch.cat([(p.grad if p.grad is not None else torch.zeros_like(p)).reshape(-1)
                      for p in net.parameters()])


# --------------------------------------------------------------------------
# Differential operators (base/diff_ops.py)
# --------------------------------------------------------------------------
def op_gradient(y, x, grad_outputs=None):
    """d(sum_c g_c y_c)/dx with create_graph (base/diff_ops.py:53-58)."""
    g = torch.ones_like(y) if grad_outputs is None else grad_outputs
    return torch.autograd.grad(y, [x], grad_outputs=g, create_graph=True)[0]


def op_divergence(y, x):
    """sum_i dy_i/dx_i, one reverse pass per channel (base/diff_ops.py:44-50)."""
    acc = 0.0
    for i in range(y.shape[-1]):
        yi = y[..., i]
        gi = torch.autograd.grad(yi, x, torch.ones_like(yi), create_graph=True)[0]
        acc = acc + gi[..., i:i + 1]
    return acc


def op_laplace(y, x):
    """div(grad y) (base/diff_ops.py:33-41, normalize=False)."""
    return op_divergence(op_gradient(y, x), x)


def op_jacobian(y, x):
    """(N, dy, dx) Jacobian plus NaN status -1/0 (base/diff_ops.py:61-82)."""
    rows = []
    for i in range(y.shape[-1]):
        yi = y[..., i]
        rows.append(torch.autograd.grad(yi, x, torch.ones_like(yi), create_graph=True)[0])
    jac = torch.stack(rows, dim=-2)
    status = -1 if bool(torch.isnan(jac).any()) else 0
    return jac, status


def op_hessian(y, x):
    """(..., dy, dx, dx) Hessian plus NaN status (base/diff_ops.py:6-30)."""
    blocks = []
    for i in range(y.shape[-1]):
        yi = y[..., i]
        gi = torch.autograd.grad(yi, x, torch.ones_like(yi), create_graph=True)[0]
        rows = []
        for j in range(x.shape[-1]):
            gij = gi[..., j]
            rows.append(torch.autograd.grad(gij, x, torch.ones_like(gij), create_graph=True)[0])
        blocks.append(torch.stack(rows, dim=-2))
    h = torch.stack(blocks, dim=-3)
    status = -1 if bool(torch.isnan(h).any()) else 0
    return h, status


# --------------------------------------------------------------------------
# Samplers (base/sampling.py) -- explicit generator so tests are seeded
# --------------------------------------------------------------------------
def sample_random(n, sdim, generator=None):
    """U[-1,1)^sdim (base/sampling.py:14-18)."""
    return torch.rand(n, sdim, generator=generator) * 2 - 1


def sample_uniform(resolution, sdim):
    """Cell-centred grid (i+0.5)/R*2-1, ij-indexed, flattened (base/sampling.py:4-11)."""
    c = torch.linspace(0.5, resolution - 0.5, resolution) / resolution * 2 - 1
    g = torch.stack(torch.meshgrid([c] * sdim, indexing='ij'), dim=-1)
    return g.reshape(resolution ** sdim, sdim)


def sample_boundary2d_side(n, side, eps=1e-4, generator=None):
    """Two thin bands of n//2 random points each (base/sampling.py:45-64)."""
    if side == 'horizontal':
        bands = (((-1 - eps, -1 + eps), (-1, 1)), ((1 - eps, 1 + eps), (-1, 1)))
    elif side == 'vertical':
        bands = (((-1, 1), (-1 - eps, -1 + eps)), ((-1, 1), (1 - eps, 1 + eps)))
    else:
        raise RuntimeError(side)
    out = []
    for (x0, x1), (y0, y1) in bands:
        p = torch.empty(n // 2, 2)
        p[:, 0] = torch.rand(n // 2, generator=generator) * (x1 - x0) + x0
        p[:, 1] = torch.rand(n // 2, generator=generator) * (y1 - y0) + y0
        out.append(p)
    return torch.cat(out, 0)


def sample_boundary1d(n, eps=1e-4, generator=None):
    """1-D boundary bands around -1 and +1 (base/sampling.py:21-27)."""
    left = (torch.rand(n // 2, 1, generator=generator) * 2 - 1) * eps - 1.0
    right = (torch.rand(n // 2, 1, generator=generator) * 2 - 1) * eps + 1.0
    return torch.cat([left, right], 0)


# --------------------------------------------------------------------------
# Initial conditions
# --------------------------------------------------------------------------
def gaussian_like(x, mu=-1.5, sigma=0.1):
    """advection/examples.py:6-16 ('example1' -> mu=-1.5)."""
    return torch.exp(-0.5 * (x - mu) ** 2 / sigma ** 2)


def taylorgreen(samples, rescale=True):
    """fluid/examples.py:17-31 (A=a=b=1, B=-1; 'taylorgreen' rescales by 1/pi)."""
    X = (samples[..., 0] + 1) * math.pi
    Y = (samples[..., 1] + 1) * math.pi
    u = torch.sin(X) * torch.cos(Y)
    v = -torch.cos(X) * torch.sin(Y)
    if rescale:
        u, v = u / math.pi, v / math.pi
    return torch.stack([u, v], -1)


def taylorgreen_multi(samples, scale=8):
    """fluid/examples.py:34-51 -- two Taylor-Green patches blended over a gap."""
    gap = 0.05
    vel = torch.zeros_like(samples)
    m1 = (samples[..., 0] <= gap) & (samples[..., 1] <= gap)
    s1 = samples[m1]
    w1 = 1.0 - s1.clamp(min=0, max=gap).norm(dim=-1) / gap
    vel[m1] = taylorgreen(torch.clamp(s1 * 2 + 1, -1, 1), rescale=False) * w1[:, None]
    p = 1 - 2 / scale
    g2 = gap * 2 / scale
    m2 = (samples[..., 0] > p - g2) & (samples[..., 1] > p - g2)
    s2 = samples[m2]
    w2 = 1.0 - (p - s2).clamp(min=0, max=g2).norm(dim=-1) / g2
    vel[m2] = taylorgreen(torch.clamp(s2 * scale + (1 - scale), -1, 1), rescale=False) * w2[:, None]
    return vel


# --------------------------------------------------------------------------
# Phase residuals (the loss_dict each inner iteration returns)
# --------------------------------------------------------------------------
def advect1d_loss(field, field_prev, x, bc, dt, vel):
    """advection/model.py:68-91 (midpoint rule + Dirichlet bc)."""
    u0 = field_prev(x)
    u = field(x)
    dudt = (u - u0) / dt
    gu = op_gradient(u, x)
    gu0 = op_gradient(u0, x).detach()
    main = torch.mean((dudt + vel * (gu + gu0) / 2.0) ** 2)
    bcl = torch.mean(field(bc) ** 2) * 1.0
    return {'main': main, 'bc': bcl}


def advect1d_init_loss(field, x, init_fn=gaussian_like):
    """advection/model.py:43-52."""
    return {'main': torch.nn.functional.mse_loss(field(x), init_fn(x))}


def fluid_init_loss(vel, x, init_fn=taylorgreen):
    """fluid/model.py:42-51."""
    return {'main': torch.nn.functional.mse_loss(vel(x), init_fn(x))}


def fluid_advect_loss(vel, vel_prev, x, bcx, bcy, dt):
    """fluid/model.py:72-101 (semi-Lagrangian backtrace, clamped to the box)."""
    with torch.no_grad():
        u_prev = vel_prev(x).detach()
    u = vel(x)
    back = torch.clamp(x - u_prev * dt, min=-1.0, max=1.0)
    with torch.no_grad():
        u_adv = vel_prev(back).detach()
    main = torch.mean((u - u_adv) ** 2)
    bcl = (torch.mean(vel(bcx)[..., 0] ** 2) + torch.mean(vel(bcy)[..., 1] ** 2)) * 1.0
    return {'main': main, 'bc': bcl}


def fluid_pressure_loss(vel, pres, x, bcx, bcy):
    """fluid/model.py:103-125: (div u - lap p)^2 + Neumann bc."""
    div_u = op_divergence(vel(x), x).detach()
    lap_p = op_laplace(pres(x), x)
    main = torch.mean((div_u - lap_p) ** 2)
    gpx = op_gradient(pres(bcx), bcx)[..., 0]
    gpy = op_gradient(pres(bcy), bcy)[..., 1]
    return {'main': main, 'bc': torch.mean(gpx ** 2) + torch.mean(gpy ** 2)}


def fluid_projection_loss(vel, vel_prev, pres, x, bcx, bcy):
    """fluid/model.py:127-151: u <- u_prev - grad p."""
    with torch.no_grad():
        u_prev = vel_prev(x).detach()
    gp = op_gradient(pres(x), x).detach()
    main = torch.mean((vel(x) - (u_prev - gp)) ** 2)
    bcl = (torch.mean(vel(bcx)[..., 0] ** 2) + torch.mean(vel(bcy)[..., 1] ** 2)) * 1.0
    return {'main': main, 'bc': bcl}


def elasticity_init_loss(f, x):
    """elasticity/model.py:109-117."""
    return {'main': torch.mean(f(x) ** 2)}


def elasticity_loss(f, f_prev, f_pp, x, fixed_l, fixed_r, cfg, timestep=1):
    """elasticity/model.py:127-189 with losses from elasticity/losses.py:6-39.

    cfg keys: dt, energy (list), ratio_arap, ratio_volume, ratio_kinematics,
    ratio_constraint, ratio_collide, plane_height, external_force (d,),
    constraint_offset_right (d,), circle_center (d,), circle_radius,
    external_force_timesteps.
    """
    dt = cfg['dt']
    with torch.no_grad():
        q_prev = f_prev(x) + x
        q_pp = f_pp(x) + x
    q = f(x) + x
    qdot = (q - q_prev) / dt
    qdot_prev = (q_prev - q_pp) / dt
    jac, _ = op_jacobian(q, x)
    S = torch.linalg.svdvals(jac)
    e_arap = cfg['ratio_arap'] * torch.sum((S - 1.0) ** 2)
    e_vol = cfg['ratio_volume'] * torch.sum((torch.prod(S, dim=1) - 1) ** 2)
    e_kin = cfg['ratio_kinematics'] * torch.sum((qdot - qdot_prev) ** 2)
    fext = torch.as_tensor(cfg['external_force'], dtype=x.dtype)
    e_ext = -dt * torch.sum(qdot * fext)
    loss = 0
    for name in cfg['energy']:
        if name == 'arap':
            loss = loss + e_arap
        elif name == 'volume':
            loss = loss + e_vol
        elif name == 'kinematics':
            loss = loss + e_kin
        elif name == 'external':
            if timestep <= cfg['external_force_timesteps']:
                loss = loss + e_ext
        elif name == 'constraint':
            loss = loss + cfg['ratio_constraint'] * torch.sum(f(fixed_l) ** 2)
        elif name == 'constraint_right':
            tgt = torch.as_tensor(cfg['constraint_offset_right'], dtype=x.dtype)
            loss = loss + cfg['ratio_constraint'] * torch.sum((f(fixed_r) - tgt) ** 2)
        elif name == 'constraint_right_compress':
            tgt = torch.as_tensor(cfg['constraint_offset_right'], dtype=x.dtype)
            loss = loss + cfg['ratio_constraint'] * torch.sum((f(fixed_r) + tgt) ** 2)
        elif name == 'collision':
            loss = loss + collision_plane(q, qdot, dt, cfg['ratio_collide'], cfg['plane_height'])
        elif name == 'collision_sphere':
            loss = loss + collision_sphere(q, qdot, dt, cfg['ratio_collide'],
                                           torch.as_tensor(cfg['circle_center'], dtype=x.dtype),
                                           cfg['circle_radius'])
        else:
            raise NotImplementedError(name)
    return {'main': loss}


def collision_plane(q, qdot, dt, ratio, height):
    """elasticity/losses.py:10-20: penalty force on points below the plane."""
    hit = q[:, -1] < height
    if int(hit.sum()) == 0:
        return 0
    depth = height - q[hit][:, -1]
    force = torch.zeros_like(q[hit])
    force[:, -1] = ratio * depth
    return -dt * torch.sum(qdot[hit] * force)


def collision_sphere(q, qdot, dt, ratio, center, radius):
    """elasticity/losses.py:22-39: penalty force on points inside the sphere."""
    vec = q - center
    dist = torch.sqrt(torch.sum(vec ** 2, dim=1))
    direc = vec / dist[:, None]
    hit = dist < radius
    if int(hit.sum()) == 0:
        return 0
    if q.shape[1] == 2:
        force = ratio * dist[hit][:, None] * direc[hit]
    else:  # losses.py:35: dist[:, None, None] * dir broadcasts to (K, K, 3), as in the reference
        force = ratio * dist[hit][:, None, None] * direc[hit]
    return -dt * torch.sum(qdot[hit] * force)


# --------------------------------------------------------------------------
# Optimiser (torch.optim.Adam single-tensor path, torch 2.x) + LR schedule
# --------------------------------------------------------------------------
class OracleAdam:
    """Adam(betas=(0.9,0.999), eps=1e-8, wd=0) as built by base/baseModel.py:55-60.

    Per element, same op order as torch's single-tensor Adam:
      m <- lerp(m, g, 1-b1);  v <- v*b2 + (1-b2) g*g
      p <- p - (lr/(1-b1^t)) * m / (sqrt(v)/sqrt(1-b2^t) + eps)
    """

    def __init__(self, params, lr, betas=(0.9, 0.999), eps=1e-8):
        self.params = list(params)
        self.lr = lr
        self.b1, self.b2 = betas
        self.eps = eps
        self.t = 0
        self.m = [torch.zeros_like(p) for p in self.params]
        self.v = [torch.zeros_like(p) for p in self.params]

    @torch.no_grad()
    def step(self):
        self.t += 1
        bc1 = 1 - self.b1 ** self.t
        bc2s = math.sqrt(1 - self.b2 ** self.t)
        for p, m, v in zip(self.params, self.m, self.v):
            if p.grad is None:
                continue
            g = p.grad
            m.lerp_(g, 1 - self.b1)
            v.mul_(self.b2).addcmul_(g, g, value=1 - self.b2)
            denom = (v.sqrt() / bc2s).add_(self.eps)
            p.addcdiv_(m, denom, value=-(self.lr / bc1))


class OraclePlateau:
    """ReduceLROnPlateau(mode=min, rel threshold 1e-4, cooldown 0, eps 1e-8)
    with the factor/patience/min_lr of base/baseModel.py:55-62."""

    def __init__(self, lr, factor=0.1, patience=500, min_lr=1e-8, threshold=1e-4, eps=1e-8):
        self.lr, self.factor, self.patience = lr, factor, patience
        self.min_lr, self.threshold, self.eps = min_lr, threshold, eps
        self.best = math.inf
        self.bad = 0

    def step(self, metric):
        metric = float(metric)
        if metric < self.best * (1.0 - self.threshold):
            self.best, self.bad = metric, 0
        else:
            self.bad += 1
        if self.bad > self.patience:
            new = max(self.lr * self.factor, self.min_lr)
            if self.lr - new > self.eps:
                self.lr = new
            self.bad = 0
        return self.lr


def update_step(nets, loss_dict, opt):
    """base/baseModel.py:73-81: sum losses, zero grads, backward, Adam step."""
    loss = sum(loss_dict.values())
    for n in nets:
        for p in n.parameters():
            p.grad = None
    loss.backward()
    opt.step()
    return loss
