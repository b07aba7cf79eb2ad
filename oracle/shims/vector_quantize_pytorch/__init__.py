"""Restatement of vector_quantize_pytorch 1.17.8 ResidualFSQ (inference path used by the
reference decoder: get_output_from_indices)."""
import torch


class FSQ(torch.nn.Module):
    def __init__(self, levels):
        super().__init__()
        lv = torch.tensor(levels, dtype=torch.int32)
        self.register_buffer("_levels", lv, persistent=False)
        basis = torch.cumprod(torch.tensor([1] + list(levels[:-1])), dim=0, dtype=torch.int32)
        self.register_buffer("_basis", basis, persistent=False)
        self.codebook_size = int(torch.prod(lv))
        self.register_buffer("implicit_codebook", self._indices_to_codes(torch.arange(self.codebook_size)),
                             persistent=False)

    def _indices_to_codes(self, indices):
        level_indices = (indices[..., None] // self._basis) % self._levels
        half_width = self._levels // 2
        return (level_indices - half_width) / half_width


class ResidualFSQ(torch.nn.Module):
    def __init__(self, *, levels, num_quantizers, dim=None, **kwargs):
        super().__init__()
        codebook_dim = len(levels)
        dim = dim if dim is not None else codebook_dim
        self.project_in = torch.nn.Linear(dim, codebook_dim) if dim != codebook_dim else torch.nn.Identity()
        self.project_out = torch.nn.Linear(codebook_dim, dim) if dim != codebook_dim else torch.nn.Identity()
        self.layers = torch.nn.ModuleList([FSQ(levels) for _ in range(num_quantizers)])
        lt = torch.tensor(levels, dtype=torch.float32)
        self.register_buffer("scales", torch.stack([(lt - 1) ** -q for q in range(num_quantizers)]),
                             persistent=False)

    @property
    def codebooks(self):
        return torch.stack([layer.implicit_codebook for layer in self.layers])

    def get_codes_from_indices(self, indices):
        # indices: [b, n, q] -> codes [q, b, n, d]
        q = indices.shape[-1]
        cb = self.codebooks[:q]
        codes = torch.stack([cb[i][indices[..., i]] for i in range(q)])
        return codes * self.scales[:q].view(q, 1, 1, -1)

    def get_output_from_indices(self, indices):
        codes = self.get_codes_from_indices(indices)
        return self.project_out(codes.sum(0))


# ---- the quantize (encoder) direction, vector_quantize_pytorch 1.17.8 inference path ----
# FSQ.bound: half_l = (L - 1)(1 + eps) / 2, offset = 0.5 for even L, shift = atanh(offset /
# half_l), bounded = tanh(z + shift) * half_l - offset; quantize = round(bound(z)) / (L // 2);
# codes_to_indices: sum((codes * (L // 2) + L // 2) * basis).  ResidualFSQ.forward bounds the
# projected input once with the first quantizer's bound before the per-quantizer loop, whose
# FSQ bounds again (the HF Xcodec2 port keeps both for checkpoint consistency).


def _fsq_bound(self, z, eps=1e-3):
    levels = self._levels.to(z.dtype)
    half_l = (levels - 1) * (1 + eps) / 2
    offset = torch.where(self._levels % 2 == 0, 0.5, 0.0).to(z.dtype)
    shift = (offset / half_l).atanh()
    return (z + shift).tanh() * half_l - offset


def _fsq_forward(self, z):
    z = z.float()
    half_width = (self._levels // 2).to(z.dtype)
    codes = self.bound(z).round() / half_width
    indices = ((codes * half_width + half_width) * self._basis.to(z.dtype)).sum(dim=-1).to(torch.int32)
    return codes, indices


def _rfsq_forward(self, x):
    x = self.project_in(x)
    residual = self.layers[0].bound(x)
    quantized_out = 0.0
    all_indices = []
    for layer, scale in zip(self.layers, self.scales):
        quantized, indices = layer(residual / scale)
        quantized = quantized * scale
        residual = residual - quantized.detach()
        quantized_out = quantized_out + quantized
        all_indices.append(indices)
    return self.project_out(quantized_out), torch.stack(all_indices, dim=-1)


FSQ.bound = _fsq_bound
FSQ.forward = _fsq_forward
ResidualFSQ.forward = _rfsq_forward
