"""Results schema of the Monte-Carlo sweep -- same fields and JSON/CSV layout as
python_ldpc_app/results.py (SNRPointResult :21-36, SimulationConfig :40-60,
SimulationResult.to_json / to_csv / from_json :70-117), so consumers of the
reference's output files (plot_results.py) read ours unchanged."""
import csv
import json
from dataclasses import asdict, dataclass, field, fields
from typing import List, Tuple


@dataclass
class SNRPointResult:
    snr_db: float
    ber: float
    fer: float
    avg_normalized_llr: float
    total_blocks: int
    successful_blocks: int
    failed_blocks: int
    avg_convergence_iterations: float
    matrix_path: str = ""
    modulation: int = 1
    max_iterations: int = 5
    interleaver: str = "none"
    encoding_method: str = "standard"


@dataclass
class SimulationConfig:
    matrix_path: str
    n: int
    m: int
    k: int
    rate: float
    blocks: int
    max_iterations: int
    encoding_method: str
    interleaver_type: str
    decoder_type: str
    channel_mode: int
    modulation: int
    speed: float
    snr_range: Tuple[float, float, float]
    threads: int
    timestamp: str
    interference_snr: float = 0.0
    p: float = 0.1


CSV_FIELDS = ["snr_db", "ber", "fer", "avg_normalized_llr", "total_blocks", "successful_blocks",
              "failed_blocks", "avg_convergence_iterations", "matrix_path", "modulation",
              "max_iterations", "interleaver", "encoding_method"]


@dataclass
class SimulationResult:
    config: SimulationConfig
    snr_points: List[SNRPointResult]
    wall_clock_seconds: float
    adaptation_log: List[dict] = field(default_factory=list)

    def to_dict(self):
        d = asdict(self)
        d["config"]["snr_range"] = list(d["config"]["snr_range"])
        return d

    def to_json(self, path):
        with open(path, "w", encoding="utf-8") as fh:
            json.dump(self.to_dict(), fh, indent=2, ensure_ascii=False)

    def to_csv(self, path):
        if not self.snr_points:
            return
        with open(path, "w", newline="", encoding="utf-8") as fh:
            w = csv.DictWriter(fh, fieldnames=CSV_FIELDS)
            w.writeheader()
            for sp in self.snr_points:
                w.writerow({k: getattr(sp, k) for k in CSV_FIELDS})

    @classmethod
    def from_json(cls, path):
        with open(path, "r", encoding="utf-8") as fh:
            d = json.load(fh)
        cfg = dict(d["config"])
        cfg["snr_range"] = tuple(cfg["snr_range"])
        names = {f.name for f in fields(SimulationConfig)}
        config = SimulationConfig(**{k: v for k, v in cfg.items() if k in names})
        pts = [SNRPointResult(**sp) for sp in d["snr_points"]]
        return cls(config=config, snr_points=pts, wall_clock_seconds=d["wall_clock_seconds"],
                   adaptation_log=d.get("adaptation_log", []))
