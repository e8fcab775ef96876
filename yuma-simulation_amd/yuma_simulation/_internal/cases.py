"""The 14 built-in 3-validator x 2-server scenarios (reference _internal/cases.py).

Same public surface: ``BaseCase``, ``register_case``, ``create_case``,
``class_registry``, ``Case1`` ... ``Case14`` and the ``cases`` list, with the
same names, validator labels, base validators, reset metadata and per-epoch
weights / stakes. Each case is written here as a *schedule*: a list of
(first_epoch, last_epoch, row_weights) segments, where row_weights gives every
validator's [server 1, server 2] weight. ``weights_epochs`` builds the list
once and caches it (the reference rebuilds it on every access, which made its
epoch loop O(E^2) — SURVEY §3 hot loop 3); ``packed_weights`` /
``packed_stakes`` give the [E, V, M] / [E, V] tensors the engine consumes.
"""

from __future__ import annotations

from dataclasses import dataclass, field

import torch

class_registry: dict[str, type] = {}


def register_case(name: str):
    """Class decorator adding a case class to ``class_registry`` under `name`."""

    def decorator(cls):
        class_registry[name] = cls
        return cls

    return decorator


S1 = (1.0, 0.0)  # all weight on server 1
S2 = (0.0, 1.0)  # all weight on server 2
LAST = 10**9     # open-ended segment end


def _build(num_epochs: int, segments, servers: int = 2) -> list[torch.Tensor]:
    out = []
    for epoch in range(num_epochs):
        W = torch.zeros(3, servers)
        for first, last, rows in segments:
            if first <= epoch <= last:
                W = torch.tensor([list(r) for r in rows], dtype=torch.float32)
                break
        out.append(W)
    return out


@dataclass
class BaseCase:
    name: str
    validators: list[str]
    base_validator: str
    num_epochs: int = 40
    reset_bonds: bool = False
    reset_bonds_index: int = None
    reset_bonds_epoch: int = None
    servers: list[str] = field(default_factory=lambda: ["Server 1", "Server 2"])

    # (first_epoch, last_epoch, rows) segments; subclasses override
    weight_schedule = ()
    stake_schedule = ((0, LAST, (0.8, 0.1, 0.1)),)

    def __post_init__(self):
        if self.base_validator not in self.validators:
            raise ValueError(f"base_validator '{self.base_validator}' must be in validators list.")

    @property
    def weights_epochs(self) -> list[torch.Tensor]:
        if not self.weight_schedule:
            raise NotImplementedError("Subclasses must implement the weights_epochs property.")
        return [w.clone() for w in self._cached("_w", lambda: _build(self.num_epochs, self.weight_schedule))]

    @property
    def stakes_epochs(self) -> list[torch.Tensor]:
        def make():
            out = []
            for epoch in range(self.num_epochs):
                for first, last, s in self.stake_schedule:
                    if first <= epoch <= last:
                        out.append(torch.tensor(s, dtype=torch.float32))
                        break
            return out

        return [s.clone() for s in self._cached("_s", make)]

    def _cached(self, key, make):
        store = self.__dict__.setdefault("_schedule_cache", {})
        tag = (key, self.num_epochs)
        if tag not in store:
            store[tag] = make()
        return store[tag]

    def packed_weights(self) -> torch.Tensor:
        """[E, V, M] float32 weights (one build, no per-epoch rebuild)."""
        return torch.stack(self.weights_epochs)

    def packed_stakes(self) -> torch.Tensor:
        """[E, V] float32 stakes."""
        return torch.stack(self.stakes_epochs)

    def packed_inputs(self) -> tuple[torch.Tensor, torch.Tensor]:
        """([E, V, M] weights, [E, V] stakes) of the first num_epochs epochs,
        built once per case and shared: read-only (run_simulations stacks them
        into the engine's batch; the public *_epochs properties keep handing
        out fresh copies as the reference does)."""
        def make():
            E = self.num_epochs
            W = torch.stack(list(self.weights_epochs)[:E]).to(torch.float32)
            S = torch.stack(list(self.stakes_epochs)[:E]).to(torch.float32)
            return W, S

        return self._cached("_packed", make)


def create_case(case_name: str, **kwargs) -> BaseCase:
    if case_name not in class_registry:
        raise ValueError(f"Case '{case_name}' is not registered.")
    return class_registry[case_name](**kwargs)


def _vals(*names):
    return field(default_factory=lambda: list(names))


@register_case("Case 1")
@dataclass
class Case1(BaseCase):
    name: str = "Case 1 - kappa moves first"
    validators: list[str] = _vals("Big vali. (0.8)", "Small lazy vali. (0.1)", "Small lazier vali. (0.1)")
    base_validator: str = "Big vali. (0.8)"
    weight_schedule = (
        (0, 0, (S1, S1, S1)),
        (1, 1, (S2, S1, S1)),
        (2, 2, (S2, S2, S1)),
        (3, LAST, (S2, S2, S2)),
    )


@register_case("Case 2")
@dataclass
class Case2(BaseCase):
    name: str = "Case 2 - kappa moves second"
    validators: list[str] = _vals("Big vali. (0.8)", "Small eager vali. (0.1)", "Small lazy vali. (0.1)")
    base_validator: str = "Small eager vali. (0.1)"
    weight_schedule = (
        (0, 0, (S1, S1, S1)),
        (1, 1, (S1, S2, S1)),
        (2, 2, (S2, S2, S1)),
        (3, LAST, (S2, S2, S2)),
    )


@register_case("Case 3")
@dataclass
class Case3(BaseCase):
    name: str = "Case 3 - kappa moves third"
    validators: list[str] = _vals("Big vali. (0.8)", "Small eager vali. (0.1)", "Small lazy vali. (0.1)")
    base_validator: str = "Small eager vali. (0.1)"
    weight_schedule = (
        (0, 0, (S1, S1, S1)),
        (1, 1, (S1, S2, S1)),
        (2, 2, (S1, S2, S2)),
        (3, LAST, (S2, S2, S2)),
    )


@register_case("Case 4")
@dataclass
class Case4(BaseCase):
    name: str = "Case 4 - all validators switch"
    validators: list[str] = _vals("Big vali. (0.8)", "Small vali. (0.1)", "Small vali 2. (0.1)")
    base_validator: str = "Big vali. (0.8)"
    weight_schedule = (
        (0, 0, (S1, S1, S1)),
        (1, LAST, (S2, S2, S2)),
    )


@register_case("Case 5")
@dataclass
class Case5(BaseCase):
    name: str = "Case 5 - kappa moves second, then third"
    validators: list[str] = _vals("Big vali. (0.8)", "Small eager-eager vali. (0.1)", "Small eager-lazy vali. (0.1)")
    base_validator: str = "Small eager-eager vali. (0.1)"
    reset_bonds: bool = True
    reset_bonds_index: int = 1
    reset_bonds_epoch: int = 20
    weight_schedule = (
        (0, 0, (S1, S1, S1)),
        (1, 1, (S1, S2, S2)),
        (2, 20, (S2, S2, S2)),
        (21, 21, (S2, S1, S2)),
        (22, 22, (S2, S1, S1)),
        (23, LAST, (S1, S1, S1)),
    )


@register_case("Case 6")
@dataclass
class Case6(BaseCase):
    name: str = "Case 6 - kappa moves second, then all validators switch"
    validators: list[str] = _vals("Big vali. (0.8)", "Small eager vali. (0.1)", "Small lazy vali. (0.1)")
    base_validator: str = "Small eager vali. (0.1)"
    reset_bonds: bool = True
    reset_bonds_index: int = 0
    reset_bonds_epoch: int = 21
    weight_schedule = (
        (0, 0, (S1, S1, S1)),
        (1, 1, (S1, S2, S1)),
        (2, 2, (S2, S2, S1)),
        (3, 20, (S2, S2, S2)),
        (21, LAST, (S1, S1, S1)),
    )


@register_case("Case 7")
@dataclass
class Case7(BaseCase):
    name: str = "Case 7 - big vali moves late, then all but one small vali moves late"
    validators: list[str] = _vals("Big vali. (0.8)", "Small eager-lazy vali. (0.1)", "Small eager-eager vali. (0.1)")
    base_validator: str = "Small eager-eager vali. (0.1)"
    reset_bonds: bool = True
    reset_bonds_index: int = 0
    reset_bonds_epoch: int = 21
    weight_schedule = (
        (0, 0, (S1, S1, S1)),
        (1, 1, (S1, S2, S2)),
        (2, 20, (S2, S2, S2)),
        (21, 21, (S2, S2, S1)),
        (22, LAST, (S1, S1, S1)),
    )


@register_case("Case 8")
@dataclass
class Case8(BaseCase):
    name: str = "Case 8 - big vali moves late, then late"
    validators: list[str] = _vals("Big dishonest lazy vali. (0.8)", "Small eager-eager vali. (0.1)", "Small eager-eager vali 2. (0.1)")
    base_validator: str = "Small eager-eager vali. (0.1)"
    reset_bonds: bool = True
    reset_bonds_index: int = 1
    reset_bonds_epoch: int = 20
    weight_schedule = (
        (0, 0, (S1, S1, S1)),
        (1, 1, (S1, S2, S2)),
        (2, 20, (S2, S2, S2)),
        (21, 21, (S2, S1, S1)),
        (22, LAST, (S1, S1, S1)),
    )


@register_case("Case 9")
@dataclass
class Case9(BaseCase):
    name: str = "Case 9 - small validators merged in e5"
    validators: list[str] = _vals("Big vali. (0.8)", "Small vali. (0.1/0.2)", "Small vali 2. (0.1/0.0)")
    base_validator: str = "Big vali. (0.8)"
    weight_schedule = ((0, LAST, (S2, S2, S2)),)
    stake_schedule = (
        (0, 5, (0.8, 0.1, 0.1)),
        (6, LAST, (0.8, 0.2, 0.0)),
    )


@register_case("Case 10")
@dataclass
class Case10(BaseCase):
    name: str = "Case 10 - kappa delayed"
    validators: list[str] = _vals("Big delayed vali. (0.8)", "Small eager vali. (0.1)", "Small lazy vali. (0.1)")
    base_validator: str = "Small eager vali. (0.1)"
    weight_schedule = (
        (0, 0, (S1, S1, S1)),
        (1, 9, (S1, S2, S1)),
        (10, 10, (S2, S2, S1)),
        (11, LAST, (S2, S2, S2)),
    )


@register_case("Case 11")
@dataclass
class Case11(BaseCase):
    name: str = "Case 11 - clipping demo"
    validators: list[str] = _vals("Big vali. 1 (0.49)", "Big vali. 2 (0.49)", "Small vali. (0.02)")
    base_validator: str = "Big vali. 1 (0.49)"
    reset_bonds: bool = True
    reset_bonds_index: int = 1
    reset_bonds_epoch: int = 20
    weight_schedule = (
        (0, 19, ((0.3, 0.7), (0.6, 0.4), (0.61, 0.39))),
        (20, LAST, ((0.3, 0.7), (0.6, 0.4), (0.3, 0.61))),
    )
    stake_schedule = ((0, LAST, (0.49, 0.49, 0.02)),)


@register_case("Case 12")
@dataclass
class Case12(BaseCase):
    name: str = "Case 12 - all validators switch, but small validator/s support alt miner with minimal weight"
    validators: list[str] = _vals("Big vali. (0.8)", "Small dishonest vali. (0.1)", "Small vali. (0.1)")
    base_validator: str = "Big vali. (0.8)"
    reset_bonds: bool = True
    reset_bonds_index: int = 1
    reset_bonds_epoch: int = 20
    weight_schedule = (
        (0, 0, (S1, (0.999, 0.001), S1)),
        (1, 20, (S2, (0.001, 0.999), S2)),
        (21, LAST, (S1, (0.999, 0.001), S1)),
    )


@register_case("Case 13")
@dataclass
class Case13(BaseCase):
    name: str = "Case 13 - Big vali supports server 2, small validator/s support server 1"
    validators: list[str] = _vals("Big vali. (0.8)", "Small vali. (0.1)", "Small vali 2. (0.1)")
    base_validator: str = "Big vali. (0.8)"
    reset_bonds: bool = True
    reset_bonds_index: int = 0
    reset_bonds_epoch: int = 20
    weight_schedule = (
        (0, 20, (S2, (0.5, 0.5), S2)),
        (21, LAST, (S2, (0.5, 0.5), (0.5, 0.5))),
    )


@register_case("Case 14")
@dataclass
class Case14(BaseCase):
    name: str = "Case 14 - All validators support Server 1, one of them switches to Server 2 for one epoch"
    validators: list[str] = _vals("Vali. 1 (0.33)", "Vali. 2 (0.33)", "Vali. 3 (0.34)")
    base_validator: str = "Vali. 1 (0.33)"
    reset_bonds: bool = False
    weight_schedule = (
        (0, 19, (S1, S1, S1)),
        (20, 20, (S1, S1, S2)),
        (21, LAST, (S1, S1, S1)),
    )
    stake_schedule = ((0, LAST, (0.33, 0.33, 0.34)),)


cases = [cls() for cls in class_registry.values()]
