"""Trajectory export: SaveTrajectoryToCSV (towr/src/utils/save_data.cpp:9-130) on top of the engine.

The samples come from the device (`TowrGpuProblem.sample_trajectory`, the towr_traj_kernel); this
module only names the columns and writes the reference's CSV text: the same header, `std::fixed`
with 6 decimals, `is_contact_phase_i` as 0/1.
"""
from __future__ import annotations

from typing import List

import numpy as np

BASE_COLUMNS = ["time",
                "base_pos_x", "base_pos_y", "base_pos_z",
                "base_vel_x", "base_vel_y", "base_vel_z",
                "base_acc_x", "base_acc_y", "base_acc_z",
                "base_euler_roll", "base_euler_pitch", "base_euler_yaw",
                "base_omega_x", "base_omega_y", "base_omega_z",
                "base_omegadot_x", "base_omegadot_y", "base_omegadot_z"]
EE_COLUMNS = ["ee_pos_x_{i}", "ee_pos_y_{i}", "ee_pos_z_{i}",
              "ee_vel_x_{i}", "ee_vel_y_{i}", "ee_vel_z_{i}",
              "ee_acc_x_{i}", "ee_acc_y_{i}", "ee_acc_z_{i}",
              "ee_euler_roll_{i}", "ee_euler_pitch_{i}", "ee_euler_yaw_{i}",
              "ee_omega_x_{i}", "ee_omega_y_{i}", "ee_omega_z_{i}",
              "ee_omegadot_x_{i}", "ee_omegadot_y_{i}", "ee_omegadot_z_{i}",
              "contact_force_x_{i}", "contact_force_y_{i}", "contact_force_z_{i}",
              "contact_torque_x_{i}", "contact_torque_y_{i}", "contact_torque_z_{i}",
              "is_contact_phase_{i}"]


def csv_header(n_ee: int) -> List[str]:
    """Column names of save_data.cpp:27-47 (19 + 25 n_ee)."""
    cols = list(BASE_COLUMNS)
    for i in range(n_ee):
        cols += [c.format(i=i) for c in EE_COLUMNS]
    return cols


def format_csv(rows: np.ndarray, n_ee: int) -> str:
    """The CSV text SaveTrajectoryToCSV writes for these sample rows."""
    contact = {19 + 25 * i + 24 for i in range(n_ee)}
    lines = [",".join(csv_header(n_ee))]
    for r in rows:
        lines.append(",".join(str(int(v)) if j in contact else f"{v:.6f}" for j, v in enumerate(r)))
    return "\n".join(lines) + "\n"


def save_trajectory_csv(problem, x, filename: str, T_sample: float = 0.001) -> int:
    """SaveTrajectoryToCSV(solution, filename, T_sample) for the solution x of `problem`
    (a TowrGpuProblem). Returns the number of samples written."""
    rows = problem.sample_trajectory(x, T_sample)
    n_ee = (rows.shape[1] - 19) // 25
    with open(filename, "w") as fh:
        fh.write(format_csv(rows, n_ee))
    return rows.shape[0]
