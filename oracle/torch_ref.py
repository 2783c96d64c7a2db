"""torch restatement of the reference algorithm as written -- TEST INFRASTRUCTURE ONLY.

* ``elbo_naive``: reference ``compute_loss`` (mpvae.py:145-210) with the same
  tensor program -- the (S,B,L,L) pairwise ranking tensor of
  ``build_multi_classification_loss`` (mpvae.py:103-123) and autograd for the
  backward.  It is the CPU baseline of bench.py (the reference itself cannot
  travel to the GPU box) and a second checker of the golden vectors.
* ``vae_forward_reference_order``: ``VAE.forward`` (mpvae.py:86-100) on a
  module's weights, drawing dropout masks and reparameterisation noise in the
  reference's order -- the checker of the build's fused-reparam forward.
"""
import torch
import torch.nn.functional as F


def ranking_loss_pairwise(E, y):
    """mpvae.py:103-123: mean over (s,b) of sum_{pos j, neg k} e^{-5(E_j-E_k)}/(5 n)."""
    pos = y == 1.0
    neg = y == 0.0
    mask = (pos.unsqueeze(2) & neg.unsqueeze(1)).float()           # (B,L,L) [j,k]
    pair = torch.exp(-5.0 * (E.unsqueeze(3) - E.unsqueeze(2))) * mask
    n = pos.float().sum(1) * neg.float().sum(1)
    per = pair.sum(dim=(2, 3)) / (5.0 * n)
    per = torch.where(torch.isnan(per) | torch.isinf(per), torch.zeros_like(per), per)
    return per.mean()


def elbo_naive(y, fe_out, fe_mu, fe_logvar, fx_out, fx_mu, fx_logvar, R, noise, nll_coeff,
               c_coeff):
    """Returns the 8-tuple of compute_loss for an explicit noise tensor (S,B,z)."""
    kl = (0.5 * ((fx_logvar - fe_logvar) - 1 + torch.exp(fe_logvar - fx_logvar)
                 + (fx_mu - fe_mu) ** 2 / (torch.exp(fx_logvar) + 1e-6)).sum(1)).mean()
    Bt = R.t().float()
    delta = torch.tensor([1e-6], dtype=torch.float32, device=y.device)
    std_normal = torch.distributions.Normal(torch.tensor([0.0], device=y.device),
                                            torch.tensor([1.0], device=y.device))
    t = torch.tensordot(noise, Bt, dims=1)

    def branch(mean):
        E = std_normal.cdf(t + mean) * (1 - delta) + delta * 0.5
        logp = (torch.log(E) * y + torch.log(1 - E) * (1 - y)).sum(2)
        m = logp.max(0)[0]
        nll = (-torch.log(torch.exp(logp - m).mean(0)) - m).mean()
        return E, nll, ranking_loss_pairwise(E, y)

    E, nll, c = branch(fe_out)
    Ex, nll_x, c_x = branch(fx_out)
    total = (nll + nll_x) * nll_coeff + (c + c_x) * c_coeff + kl * 1.1
    return total, nll, nll_x, c, c_x, kl, Ex.mean(0), E.mean(0)


def vae_forward_reference_order(model, label, feature):
    """VAE.forward of mpvae.py:86-100 with the reference's RNG order, on the
    weights of ``model`` (any module with the reference's layer names)."""
    drop = lambda x: F.dropout(x, p=model.dropout.p, training=model.training)
    sc = model.scale_coeff

    def dec(z, head):
        return head(F.relu(model.fd2(F.relu(model.fd1(z)))))

    h = drop(F.relu(model.fe1(torch.cat((feature, label), 1))))
    h = drop(F.relu(model.fe2(h)))
    mu_e, lv_e = model.fe_mu(h) * sc, model.fe_logvar(h) * sc
    std = torch.exp(0.5 * lv_e)
    z_e = mu_e + torch.randn_like(std) * std
    label_out = dec(torch.cat((feature, z_e), 1), model.label_mp_mu)
    h = drop(F.relu(model.fx1(feature)))
    h = drop(F.relu(model.fx2(h)))
    h = drop(F.relu(model.fx3(h)))
    mu_x, lv_x = model.fx_mu(h) * sc, model.fx_logvar(h) * sc
    std = torch.exp(0.5 * lv_x)
    z_x = mu_x + torch.randn_like(std) * std
    feat_out = dec(torch.cat((feature, z_x), 1), model.feat_mp_mu)
    return label_out, mu_e, lv_e, feat_out, mu_x, lv_x
