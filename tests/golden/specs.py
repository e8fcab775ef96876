"""Configurations the golden fixtures were captured with (shared by
make_golden.py and the tests; plain data, importable without the reference)."""

VERSIONS = [
    "Yuma 0 (subtensor)", "Yuma 1 (paper)", "Yuma 1 (paper) - liquid alpha on",
    "Yuma 2 (Adrian-Fish)", "Yuma 3 (Rhef)", "Yuma 3.1 (Rhef+reset)",
    "Yuma 3.2 (Rhef+conditional)", "Yuma 4 (Rhef+relative bonds)",
    "Yuma 4 (Rhef+relative bonds) - liquid alpha on",
]
BETAS = [0, 0.5, 0.99, 1.0]

# YumaParams overrides of each sheet version (sheet script :25-48)
SHEET_PARAMS = [
    {}, {}, {"liquid_alpha": True}, {}, {}, {}, {}, {},
    {"bond_alpha": 0.025, "alpha_high": 0.99, "alpha_low": 0.9, "liquid_alpha": True},
]

VARIANTS = ["rust", "yuma1", "yuma2", "yuma3", "yuma4"]

CONFIGS = {
    "default": dict(),
    "beta05": dict(bond_penalty=0.5, kappa=0.6),
    "liquid": dict(liquid_alpha=True),
    "liquid_y4": dict(liquid_alpha=True, bond_alpha=0.025, alpha_high=0.99, alpha_low=0.9),
    "liquid_ovr_hi": dict(liquid_alpha=True, override_consensus_high=0.02),
    "liquid_ovr_lo": dict(liquid_alpha=True, override_consensus_low=0.001),
    "liquid_ovr_both": dict(liquid_alpha=True, override_consensus_high=0.03, override_consensus_low=0.002),
    "liquid_ovr_eq": dict(liquid_alpha=True, override_consensus_high=0.01, override_consensus_low=0.01),
    "precision": dict(consensus_precision=1000, kappa=0.3),
}
SIM_KEYS = {"kappa", "bond_penalty", "consensus_precision"}

LARGE_SPECS = {
    "rust": {}, "yuma1": {}, "yuma2": {}, "yuma3": {}, "yuma4": {},
    "yuma4_liquid": dict(liquid_alpha=True, bond_alpha=0.025, alpha_high=0.99, alpha_low=0.9),
    "yuma1_liquid": dict(liquid_alpha=True),
}
LARGE_SEED = 0x5EED0002
SMALL_SYNTH_SEED = 0x5EED0101
MEDIUM_SYNTH_SEED = 0x5EED0201


def split_spec(spec: dict):
    sim = {k: v for k, v in spec.items() if k in SIM_KEYS}
    par = {k: v for k, v in spec.items() if k not in SIM_KEYS}
    return sim, par
