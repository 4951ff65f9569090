"""Write the hand-made URDF fixtures of the on-GPU rigid-body model (the CENTAURO
URDF the reference loads, QPPVMPlugin.cpp:50-51, is not in the container):

* quadruped.urdf -- the ForceAcc robot: a ``pelvis`` root (floating base when loaded with
  floating_base=True), four 6-joint legs (hip yaw / roll / pitch, knee, ankle pitch / roll; one leg
  carries a prismatic "knee slider" instead of the ankle roll, to cover prismatic joints), and the
  contact frames ``foot_fl``, ``foot_fr``, ``foot_hr``, ``foot_hl`` (ForceAcc.cpp:58) on fixed joints
  under the ankles, each with a fixed sole plate carrying mass (exercising the fixed-joint lumping);
* centauro_arms.urdf -- the QPPVM robot: a fixed ``pelvis``, ``torso_yaw``, two 7-DoF arms whose
  end links ``arm1_7`` / ``arm2_7`` carry fixed ``*_ee`` frames (the QPPVMPlugin tasks, :129-152).

Deterministic (no RNG): dimensions and masses follow simple formulas. Usage:
python tests/golden/make_urdf.py
"""
import os

HERE = os.path.dirname(os.path.abspath(__file__))


def inertial(m, xyz, ixx, iyy, izz, ixy=0.0, ixz=0.0, iyz=0.0, rpy="0 0 0"):
    return (f'    <inertial><origin xyz="{xyz}" rpy="{rpy}"/><mass value="{m:.6g}"/>'
            f'<inertia ixx="{ixx:.6g}" iyy="{iyy:.6g}" izz="{izz:.6g}" ixy="{ixy:.6g}" ixz="{ixz:.6g}" '
            f'iyz="{iyz:.6g}"/></inertial>\n')


def link(name, inert=""):
    return f'  <link name="{name}">\n{inert}  </link>\n'


def joint(name, typ, parent, child, xyz, rpy="0 0 0", axis=None, effort=None, lower=None, upper=None):
    s = f'  <joint name="{name}" type="{typ}">\n    <parent link="{parent}"/><child link="{child}"/>\n'
    s += f'    <origin xyz="{xyz}" rpy="{rpy}"/>\n'
    if axis is not None:
        s += f'    <axis xyz="{axis}"/>\n'
    if effort is not None:
        s += f'    <limit effort="{effort}" lower="{lower}" upper="{upper}" velocity="10"/>\n'
    return s + '  </joint>\n'


def quadruped():
    out = ['<?xml version="1.0"?>\n<robot name="wbq_quadruped">\n']
    out.append(link("pelvis", inertial(18.0, "0.01 0 0.02", 0.35, 0.9, 1.0, 0.01, -0.02, 0.0)))
    legs = [("fl", 0.35, 0.2), ("fr", 0.35, -0.2), ("hr", -0.35, -0.2), ("hl", -0.35, 0.2)]
    names = ["hip_yaw", "hip_roll", "hip_pitch", "knee", "ankle_pitch", "ankle_roll"]
    axes = ["0 0 1", "1 0 0", "0 1 0", "0 1 0", "0 1 0", "1 0 0"]
    for li, (leg, x, y) in enumerate(legs):
        prev = "pelvis"
        for k, (jn, ax) in enumerate(zip(names, axes)):
            cl = f"{leg}_{jn}_link"
            m = 2.5 - 0.3 * k + 0.1 * li
            L = 0.05 if k < 3 else 0.3
            xyz = f"{x} {y} -0.05" if k == 0 else ("0 0 -0.3" if k in (3, 4) else "0 0 -0.04")
            typ, axis, eff, lo, hi = "revolute", ax, 120 - 10 * k, -1.5, 1.5
            if leg == "hr" and k == 5:  # a prismatic slider in one leg
                typ, axis, eff, lo, hi = "prismatic", "0 0 1", 300, -0.05, 0.05
            out.append(joint(f"{leg}_{jn}", typ, prev, cl, xyz, rpy=f"{0.02 * k} {-0.01 * li} {0.03 * (k - li)}",
                             axis=axis, effort=eff, lower=lo, upper=hi))
            out.append(link(cl, inertial(m, f"0.01 0.005 {-L / 2:.3f}", m * L * L / 12 + 0.002,
                                         m * L * L / 12 + 0.003, 0.002 + 0.001 * k, 0.0002 * k, -0.0001, 0.0003)))
            prev = cl
        out.append(joint(f"{leg}_foot_joint", "fixed", prev, f"foot_{leg}", "0 0 -0.05", rpy="0.1 -0.05 0.2"))
        out.append(link(f"foot_{leg}", inertial(0.3, "0 0 -0.01", 0.001, 0.001, 0.0015)))
        out.append(joint(f"{leg}_sole_joint", "fixed", f"foot_{leg}", f"{leg}_sole", "0.02 0 -0.02"))
        out.append(link(f"{leg}_sole", inertial(0.2, "0.01 0 0", 0.0005, 0.0008, 0.001, rpy="0 0.3 0")))
    out.append("</robot>\n")
    return "".join(out)


def centauro_arms():
    out = ['<?xml version="1.0"?>\n<robot name="wbq_centauro_arms">\n']
    out.append(link("pelvis", inertial(20.0, "0 0 0", 0.5, 0.5, 0.5)))
    out.append(joint("torso_yaw", "revolute", "pelvis", "torso", "0 0 0.3", axis="0 0 1", effort=200, lower=-2.5,
                     upper=2.5))
    out.append(link("torso", inertial(12.0, "0.02 0 0.2", 0.4, 0.35, 0.2, 0.01, 0.0, 0.0)))
    axes = ["0 1 0", "1 0 0", "0 0 1", "0 1 0", "0 0 1", "0 1 0", "0 0 1"]
    for arm, y in ((1, 0.25), (2, -0.25)):
        prev = "torso"
        for k in range(7):
            cl = f"arm{arm}_{k + 1}"
            xyz = f"0 {y} 0.4" if k == 0 else f"0 0 {-0.12 - 0.02 * (k % 3):.2f}"
            out.append(joint(f"j_arm{arm}_{k + 1}", "revolute", prev, cl, xyz,
                             rpy=f"{0.1 * (k % 2)} {0.05 * arm} {-0.07 * k}", axis=axes[k], effort=150 - 12 * k,
                             lower=-2.0, upper=2.0))
            m = 3.0 - 0.35 * k
            out.append(link(cl, inertial(m, f"0 0.01 {-0.05 - 0.01 * k:.2f}", 0.02 + 0.003 * k, 0.02, 0.008,
                                         0.001, 0.0005 * arm, -0.0004)))
            prev = cl
        out.append(joint(f"arm{arm}_ee_joint", "fixed", prev, f"arm{arm}_ee", "0 0 -0.1", rpy="0 0.2 0"))
        out.append(link(f"arm{arm}_ee", inertial(0.5, "0 0 -0.02", 0.001, 0.001, 0.001)))
    out.append("</robot>\n")
    return "".join(out)


def main():
    for name, text in (("quadruped.urdf", quadruped()), ("centauro_arms.urdf", centauro_arms())):
        with open(os.path.join(HERE, name), "w") as f:
            f.write(text)
        print("wrote", name, len(text), "bytes")


if __name__ == "__main__":
    main()
