-- As-rigid-as-possible deformation of a regular 3-D lattice: every lattice edge keeps
-- its rest vector up to the rotation of its first end; handle nodes are pulled to their
-- targets. Declaration indices follow the reference example
-- (examples/volumetric_mesh_deformation).
local nx, ny, nz = Dim("W", 0), Dim("H", 1), Dim("D", 2)

local node   = Unknown("Offset", opt_float3, {nx, ny, nz}, 0)
local turn   = Unknown("Angle", opt_float3, {nx, ny, nz}, 1)
local lattice = Array("UrShape", opt_float3, {nx, ny, nz}, 2)
local goal   = Array("Constraints", opt_float3, {nx, ny, nz}, 3)
local goalW  = Param("w_fitSqrt", float, 4)
local stiffW = Param("w_regSqrt", float, 5)
UsePreconditioner(true)

local hasGoal = greatereq(goal(0, 0, 0)(0), -999999.9)
Energy(Select(hasGoal, goalW * (node(0, 0, 0) - goal(0, 0, 0)), 0))

local faces = { {1, 0, 0}, {-1, 0, 0}, {0, 1, 0}, {0, -1, 0}, {0, 0, 1}, {0, 0, -1} }
for _, o in ipairs(faces) do
    local a, b, c = o[1], o[2], o[3]
    local deviation = (node(0, 0, 0) - node(a, b, c)) - Rotate3D(turn(0, 0, 0), lattice(0, 0, 0) - lattice(a, b, c))
    Energy(stiffW * Select(InBounds(0, 0, 0), Select(InBounds(a, b, c), deviation, 0.0), 0.0))
end
