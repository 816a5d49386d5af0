"""
Configuration dataclasses — the drop-in surface of ShawnnnLiu/Robust-NeRF
``noisy_src/config.py:10-125``.

Every reference field keeps its name and default, so ``NeRFConfig()`` and the
reference's CLI-built configs mean the same thing here.  The MI355X build adds
only defaulted fields:

* ``ModelConfig.precision`` — ``"fp32"`` (exact fp32 MFMA, the parity mode),
  ``"bf16"`` (bf16 MFMA operands, fp32 accumulation and fp32 master weights) or
  ``"fp16"`` (BASELINE cfg #5: fp16 operands, fp32 accumulation, backward on dz
  scaled by 2^14).

Data parallelism adds no config field: under ``torchrun`` the entry points read
RANK/WORLD_SIZE from the environment and slice the shared-seed global batch
(``DataConfig.batch_size`` rays) per rank.
"""

from dataclasses import dataclass, field
from pathlib import Path
from typing import Optional, Tuple


@dataclass
class ModelConfig:
    """Reference config.py:10-24."""

    pos_freqs: int = 10
    dir_freqs: int = 4
    hidden_dim: int = 256
    num_hidden_layers: int = 8
    skips: Tuple[int, ...] = (4,)
    use_view_dirs: bool = True
    # MI355X additions
    precision: str = "fp32"


@dataclass
class RenderConfig:
    """Reference config.py:27-43."""

    near: float = 2.0
    far: float = 6.0
    num_samples: int = 64
    num_samples_fine: int = 128
    use_hierarchical: bool = True
    perturb: bool = True
    raw_noise_std: float = 0.0
    white_background: bool = True


@dataclass
class DataConfig:
    """Reference config.py:46-56."""

    scene_name: str = "lego"
    data_root: Optional[Path] = None
    img_scale: float = 0.5
    batch_size: int = 1024
    shuffle: bool = True


@dataclass
class TrainConfig:
    """Reference config.py:59-83."""

    lr: float = 5e-4
    lr_decay: int = 250
    num_iterations: int = 200000
    log_every: int = 100
    save_every: int = 10000
    val_every: int = 5000
    output_dir: Path = field(default_factory=lambda: Path("outputs"))
    experiment_name: str = "baseline"
    device: str = "cuda"
    seed: int = 42


@dataclass
class PoseOptConfig:
    """Reference config.py:86-107 (defined there, never consumed; kept for the API)."""

    enabled: bool = True
    learn_rotation: bool = True
    learn_translation: bool = True
    pose_lr: float = 1e-4
    pose_opt_delay: int = 1000
    init_mode: str = "noisy"
    rotation_noise_deg: float = 0.0
    translation_noise_pct: float = 0.0
    noise_seed: Optional[int] = None


@dataclass
class NeRFConfig:
    """Reference config.py:110-125."""

    model: ModelConfig = field(default_factory=ModelConfig)
    render: RenderConfig = field(default_factory=RenderConfig)
    data: DataConfig = field(default_factory=DataConfig)
    train: TrainConfig = field(default_factory=TrainConfig)
    pose_opt: Optional[PoseOptConfig] = None

    def __post_init__(self):
        if isinstance(self.train.output_dir, str):
            self.train.output_dir = Path(self.train.output_dir)
        if isinstance(self.data.data_root, str):
            self.data.data_root = Path(self.data.data_root)
