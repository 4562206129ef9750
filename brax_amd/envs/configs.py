"""Robot descriptions used by the bundled envs.

Physical data (masses, offsets, limits) must equal the reference's for parity;
the text is our compact one-item-per-line rendering of it.
"""

# Ant robot description (the reference's `brax/envs/ant.py:290-572`,
# re-expressed in compact text format; parsed by brax_amd.config).
ANT_CONFIG = """
bodies { name: "$ Torso" colliders { capsule { radius: 0.25 length: 0.5 end: 1 } } inertia { x: 1 y: 1 z: 1 } mass: 10 }
bodies { name: "Aux 1" colliders { rotation { x: 90 y: -45 } capsule { radius: 0.08 length: 0.44284272 } } inertia { x: 1 y: 1 z: 1 } mass: 1 }
bodies { name: "$ Body 4" colliders { rotation { x: 90 y: -45 } capsule { radius: 0.08 length: 0.7256854 end: -1 } } inertia { x: 1 y: 1 z: 1 } mass: 1 }
bodies { name: "Aux 2" colliders { rotation { x: 90 y: 45 } capsule { radius: 0.08 length: 0.44284272 } } inertia { x: 1 y: 1 z: 1 } mass: 1 }
bodies { name: "$ Body 7" colliders { rotation { x: 90 y: 45 } capsule { radius: 0.08 length: 0.7256854 end: -1 } } inertia { x: 1 y: 1 z: 1 } mass: 1 }
bodies { name: "Aux 3" colliders { rotation { x: -90 y: 45 } capsule { radius: 0.08 length: 0.44284272 } } inertia { x: 1 y: 1 z: 1 } mass: 1 }
bodies { name: "$ Body 10" colliders { rotation { x: -90 y: 45 } capsule { radius: 0.08 length: 0.7256854 end: -1 } } inertia { x: 1 y: 1 z: 1 } mass: 1 }
bodies { name: "Aux 4" colliders { rotation { x: -90 y: -45 } capsule { radius: 0.08 length: 0.44284272 } } inertia { x: 1 y: 1 z: 1 } mass: 1 }
bodies { name: "$ Body 13" colliders { rotation { x: -90 y: -45 } capsule { radius: 0.08 length: 0.7256854 end: -1 } } inertia { x: 1 y: 1 z: 1 } mass: 1 }
bodies { name: "Ground" colliders { plane {  } } inertia { x: 1 y: 1 z: 1 } mass: 1 frozen { all: true } }
joints { name: "hip_1" parent_offset { x: 0.2 y: 0.2 } child_offset { x: -0.1 y: -0.1 } parent: "$ Torso" child: "Aux 1" angle_limit { min: -30 max: 30 } rotation { y: -90 } angular_damping: 20 }
joints { name: "ankle_1" parent_offset { x: 0.1 y: 0.1 } child_offset { x: -0.2 y: -0.2 } parent: "Aux 1" child: "$ Body 4" rotation { z: 135 } angle_limit { min: 30 max: 70 } angular_damping: 20 }
joints { name: "hip_2" parent_offset { x: -0.2 y: 0.2 } child_offset { x: 0.1 y: -0.1 } parent: "$ Torso" child: "Aux 2" rotation { y: -90 } angle_limit { min: -30 max: 30 } angular_damping: 20 }
joints { name: "ankle_2" parent_offset { x: -0.1 y: 0.1 } child_offset { x: 0.2 y: -0.2 } parent: "Aux 2" child: "$ Body 7" rotation { z: 45 } angle_limit { min: -70 max: -30 } angular_damping: 20 }
joints { name: "hip_3" parent_offset { x: -0.2 y: -0.2 } child_offset { x: 0.1 y: 0.1 } parent: "$ Torso" child: "Aux 3" rotation { y: -90 } angle_limit { min: -30 max: 30 } angular_damping: 20 }
joints { name: "ankle_3" parent_offset { x: -0.1 y: -0.1 } child_offset { x: 0.2 y: 0.2 } parent: "Aux 3" child: "$ Body 10" rotation { z: 135 } angle_limit { min: -70 max: -30 } angular_damping: 20 }
joints { name: "hip_4" parent_offset { x: 0.2 y: -0.2 } child_offset { x: -0.1 y: 0.1 } parent: "$ Torso" child: "Aux 4" rotation { y: -90 } angle_limit { min: -30 max: 30 } angular_damping: 20 }
joints { name: "ankle_4" parent_offset { x: 0.1 y: -0.1 } child_offset { x: -0.2 y: 0.2 } parent: "Aux 4" child: "$ Body 13" rotation { z: 45 } angle_limit { min: 30 max: 70 } angular_damping: 20 }
actuators { name: "hip_1" joint: "hip_1" strength: 350 torque {  } }
actuators { name: "ankle_1" joint: "ankle_1" strength: 350 torque {  } }
actuators { name: "hip_2" joint: "hip_2" strength: 350 torque {  } }
actuators { name: "ankle_2" joint: "ankle_2" strength: 350 torque {  } }
actuators { name: "hip_3" joint: "hip_3" strength: 350 torque {  } }
actuators { name: "ankle_3" joint: "ankle_3" strength: 350 torque {  } }
actuators { name: "hip_4" joint: "hip_4" strength: 350 torque {  } }
actuators { name: "ankle_4" joint: "ankle_4" strength: 350 torque {  } }
friction: 1
gravity { z: -9.8 }
angular_damping: -0.05
collide_include { first: "$ Torso" second: "Ground" }
collide_include { first: "$ Body 4" second: "Ground" }
collide_include { first: "$ Body 7" second: "Ground" }
collide_include { first: "$ Body 10" second: "Ground" }
collide_include { first: "$ Body 13" second: "Ground" }
dt: 0.05
substeps: 10
dynamics_mode: "pbd"
"""

# Humanoid robot description (upstream `brax/envs/humanoid.py:345-991`,
# re-expressed in compact text format).
HUMANOID_CONFIG = """
bodies { name: "torso" colliders { position {  } rotation { x: -90 } capsule { radius: 0.07 length: 0.28 } } colliders { position { z: 0.19 } capsule { radius: 0.09 length: 0.18 } } colliders { position { x: -0.01 z: -0.12 } rotation { x: -90 } capsule { radius: 0.06 length: 0.24 } } inertia { x: 1 y: 1 z: 1 } mass: 8.907463 }
bodies { name: "lwaist" colliders { position {  } rotation { x: -90 } capsule { radius: 0.06 length: 0.24 } } inertia { x: 1 y: 1 z: 1 } mass: 2.2619467 }
bodies { name: "pelvis" colliders { position { x: -0.02 } rotation { x: -90 } capsule { radius: 0.09 length: 0.32 } } inertia { x: 1 y: 1 z: 1 } mass: 6.6161942 }
bodies { name: "right_thigh" colliders { position { y: 0.005 z: -0.17 } rotation { x: -178.31532 } capsule { radius: 0.06 length: 0.46014702 } } inertia { x: 1 y: 1 z: 1 } mass: 4.751751 }
bodies { name: "right_shin" colliders { position { z: -0.15 } rotation { x: -180 } capsule { radius: 0.049 length: 0.398 end: -1 } } colliders { position { z: -0.35 } capsule { radius: 0.075 length: 0.15 end: 1 } } inertia { x: 1 y: 1 z: 1 } mass: 4.522842 }
bodies { name: "left_thigh" colliders { position { y: -0.005 z: -0.17 } rotation { x: 178.31532 } capsule { radius: 0.06 length: 0.46014702 } } inertia { x: 1 y: 1 z: 1 } mass: 4.751751 }
bodies { name: "left_shin" colliders { position { z: -0.15 } rotation { x: -180 } capsule { radius: 0.049 length: 0.398 end: -1 } } colliders { position { z: -0.35 } capsule { radius: 0.075 length: 0.15 end: 1 } } inertia { x: 1 y: 1 z: 1 } mass: 4.522842 }
bodies { name: "right_upper_arm" colliders { position { x: 0.08 y: -0.08 z: -0.08 } rotation { x: 135 y: 35.26439 z: -75 } capsule { radius: 0.04 length: 0.35712814 } } inertia { x: 1 y: 1 z: 1 } mass: 1.6610805 }
bodies { name: "right_lower_arm" colliders { position { x: 0.09 y: 0.09 z: 0.09 } rotation { x: -45 y: 35.26439 z: 15 } capsule { radius: 0.031 length: 0.33912814 } } colliders { position { x: 0.18 y: 0.18 z: 0.18 } capsule { radius: 0.04 length: 0.08 } } inertia { x: 1 y: 1 z: 1 } mass: 1.2295402 }
bodies { name: "left_upper_arm" colliders { position { x: 0.08 y: 0.08 z: -0.08 } rotation { x: -135 y: 35.26439 z: 75 } capsule { radius: 0.04 length: 0.35712814 } } inertia { x: 1 y: 1 z: 1 } mass: 1.6610805 }
bodies { name: "left_lower_arm" colliders { position { x: 0.09 y: -0.09 z: 0.09 } rotation { x: 45 y: 35.26439 z: -15 } capsule { radius: 0.031 length: 0.33912814 } } colliders { position { x: 0.18 y: -0.18 z: 0.18 } capsule { radius: 0.04 length: 0.08 } } inertia { x: 1 y: 1 z: 1 } mass: 1.2295402 }
bodies { name: "floor" colliders { plane {  } } inertia { x: 1 y: 1 z: 1 } mass: 1 frozen { all: true } }
joints { name: "abdomen_yz" parent: "torso" child: "lwaist" parent_offset { x: -0.01 z: -0.195 } child_offset { z: 0.065 } rotation { y: -90 } angle_limit { min: -45 max: 45 } angle_limit { min: -65 max: 30 } angular_damping: 30 }
joints { name: "abdomen_x" parent: "lwaist" child: "pelvis" parent_offset { z: -0.065 } child_offset { z: 0.1 } rotation { x: 90 } angle_limit { min: -35 max: 35 } angular_damping: 30 }
joints { name: "right_hip_xyz" parent: "pelvis" child: "right_thigh" parent_offset { y: -0.1 z: -0.04 } child_offset {  } rotation {  } angle_limit { min: -10 max: 10 } angle_limit { min: -30 max: 70 } angle_limit { min: -10 max: 10 } angular_damping: 30 }
joints { name: "right_knee" parent: "right_thigh" child: "right_shin" parent_offset { y: 0.01 z: -0.383 } child_offset { z: 0.02 } rotation { z: -90 } angle_limit { min: -160 max: -2 } angular_damping: 30 }
joints { name: "left_hip_xyz" parent: "pelvis" child: "left_thigh" parent_offset { y: 0.1 z: -0.04 } child_offset {  } angle_limit { min: -10 max: 10 } angle_limit { min: -30 max: 70 } angle_limit { min: -10 max: 10 } angular_damping: 30 }
joints { name: "left_knee" parent: "left_thigh" child: "left_shin" parent_offset { y: -0.01 z: -0.383 } child_offset { z: 0.02 } rotation { z: -90 } angle_limit { min: -160 max: -2 } angular_damping: 30 }
joints { name: "right_shoulder12" parent: "torso" child: "right_upper_arm" parent_offset { y: -0.17 z: 0.06 } child_offset {  } rotation { x: 135 y: 35.26439 } angle_limit { min: -85 max: 60 } angle_limit { min: -70 max: 50 } angular_damping: 30 }
joints { name: "right_elbow" parent: "right_upper_arm" child: "right_lower_arm" parent_offset { x: 0.18 y: -0.18 z: -0.18 } child_offset {  } rotation { x: 135 z: 90 } angle_limit { min: -90 max: 50 } angular_damping: 30 }
joints { name: "left_shoulder12" parent: "torso" child: "left_upper_arm" parent_offset { y: 0.17 z: 0.06 } child_offset {  } rotation { x: 45 y: -35.26439 } angle_limit { min: -60 max: 85 } angle_limit { min: -50 max: 70 } angular_damping: 30 }
joints { name: "left_elbow" parent: "left_upper_arm" child: "left_lower_arm" parent_offset { x: 0.18 y: 0.18 z: -0.18 } child_offset {  } rotation { x: 45 z: -90 } angle_limit { min: -90 max: 50 } angular_damping: 30 }
actuators { name: "abdomen_yz" joint: "abdomen_yz" strength: 350 torque {  } }
actuators { name: "abdomen_x" joint: "abdomen_x" strength: 350 torque {  } }
actuators { name: "right_hip_xyz" joint: "right_hip_xyz" strength: 350 torque {  } }
actuators { name: "right_knee" joint: "right_knee" strength: 350 torque {  } }
actuators { name: "left_hip_xyz" joint: "left_hip_xyz" strength: 350 torque {  } }
actuators { name: "left_knee" joint: "left_knee" strength: 350 torque {  } }
actuators { name: "right_shoulder12" joint: "right_shoulder12" strength: 100 torque {  } }
actuators { name: "right_elbow" joint: "right_elbow" strength: 100 torque {  } }
actuators { name: "left_shoulder12" joint: "left_shoulder12" strength: 100 torque {  } }
actuators { name: "left_elbow" joint: "left_elbow" strength: 100 torque {  } }
collide_include { first: "floor" second: "left_shin" }
collide_include { first: "floor" second: "right_shin" }
defaults { angles { name: "left_knee" angle { x: -25 y: 0 z: 0 } } angles { name: "right_knee" angle { x: -25 y: 0 z: 0 } } }
friction: 1
gravity { z: -9.81 }
angular_damping: -0.05
dt: 0.015
substeps: 8
dynamics_mode: "pbd"
"""

# HalfCheetah robot description (`brax/envs/half_cheetah.py`,
# _SYSTEM_CONFIG, re-expressed in compact text format).
HALFCHEETAH_CONFIG = """
bodies { name: "torso" colliders { rotation { y: 90 } capsule { radius: 0.046 length: 1.092 } } colliders { position { x: 0.6 z: 0.1 } rotation { y: 49.84733 } capsule { radius: 0.046 length: 0.392 } } inertia { x: 0.944797 y: 0.944797 z: 0.944797 } mass: 9.457333 }
bodies { name: "bthigh" colliders { position { x: 0.1 z: -0.13 } rotation { x: -180 y: 37.72396 z: -180 } capsule { radius: 0.046 length: 0.382 } } inertia { x: 0.02963628 y: 0.02963628 z: 0.02963628 } mass: 2.335527 }
bodies { name: "bshin" colliders { position { x: -0.14 z: -0.07 } rotation { x: 180 y: -63.689568 z: 180 } capsule { radius: 0.046 length: 0.392 } } inertia { x: 0.032029107 y: 0.032029107 z: 0.032029107 } mass: 2.402003 }
bodies { name: "bfoot" colliders { position { x: 0.03 z: -0.097 } rotation { y: -15.46986 } capsule { radius: 0.046 length: 0.28 } } inertia { x: 0.011705612 y: 0.011705612 z: 0.011705612 } mass: 1.6574708 }
bodies { name: "fthigh" colliders { position { x: -0.07 z: -0.12 } rotation { y: 29.793806 } capsule { radius: 0.046 length: 0.358 } } inertia { x: 0.024391336 y: 0.024391336 z: 0.024391336 } mass: 2.1759844 }
bodies { name: "fshin" colliders { position { x: 0.065 z: -0.09 } rotation { y: -34.37747 } capsule { radius: 0.046 length: 0.304 } } inertia { x: 0.014954625 y: 0.014954625 z: 0.014954625 } mass: 1.8170134 }
bodies { name: "ffoot" colliders { position { x: 0.045 z: -0.07 } rotation { y: -34.37747 } capsule { radius: 0.046 length: 0.232 } } inertia { x: 0.0067111105 y: 0.0067111105 z: 0.0067111105 } mass: 1.3383855 }
bodies { name: "floor" colliders { plane {  } } inertia { x: 1 y: 1 z: 1 } frozen { position { x: 1 y: 1 z: 1 } rotation { x: 1 y: 1 z: 1 } } }
joints { name: "bthigh" parent: "torso" child: "bthigh" parent_offset { x: -0.5 } child_offset {  } rotation { z: 90 } angle_limit { min: -29.793806 max: 60.16057 } }
joints { name: "bshin" parent: "bthigh" child: "bshin" parent_offset { x: 0.16 z: -0.25 } child_offset {  } rotation { z: 90 } angle_limit { min: -44.97719 max: 44.97719 } }
joints { name: "bfoot" parent: "bshin" child: "bfoot" parent_offset { x: -0.28 z: -0.14 } child_offset {  } rotation { z: 90 } angle_limit { min: -22.918312 max: 44.97719 } }
joints { name: "fthigh" parent: "torso" child: "fthigh" parent_offset { x: 0.5 } child_offset {  } rotation { z: 90 } angle_limit { min: -57.29578 max: 40.107044 } }
joints { name: "fshin" parent: "fthigh" child: "fshin" parent_offset { x: -0.14 z: -0.24 } child_offset {  } rotation { z: 90 } angle_limit { min: -68.75494 max: 49.84733 } }
joints { name: "ffoot" parent: "fshin" child: "ffoot" parent_offset { x: 0.13 z: -0.18 } child_offset {  } rotation { z: 90 } angle_limit { min: -28.64789 max: 28.64789 } }
actuators { name: "bthigh" joint: "bthigh" strength: 120 torque {  } }
actuators { name: "bshin" joint: "bshin" strength: 90 torque {  } }
actuators { name: "bfoot" joint: "bfoot" strength: 60 torque {  } }
actuators { name: "fthigh" joint: "fthigh" strength: 120 torque {  } }
actuators { name: "fshin" joint: "fshin" strength: 60 torque {  } }
actuators { name: "ffoot" joint: "ffoot" strength: 30 torque {  } }
friction: 0.7745967
gravity { z: -9.81 }
angular_damping: -0.01
collide_include { first: "floor" second: "torso" }
collide_include { first: "floor" second: "bfoot" }
collide_include { first: "floor" second: "ffoot" }
collide_include { first: "floor" second: "bthigh" }
collide_include { first: "floor" second: "fthigh" }
collide_include { first: "floor" second: "bshin" }
collide_include { first: "floor" second: "fshin" }
collide_include { first: "bfoot" second: "ffoot" }
dt: 0.05
substeps: 16
frozen { position { y: 1 } rotation { x: 1 z: 1 } }
dynamics_mode: "pbd"
"""
