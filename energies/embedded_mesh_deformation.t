-- Embedded deformation (same energy as the reference's
-- examples/embedded_mesh_deformation; same declaration indices): every node carries an
-- affine 3x3 matrix kept close to a rotation, neighbouring nodes predict each other's
-- positions through it, and handles pull nodes to their targets.
local N = Dim("N", 0)
local NUMEDGES = Dim("NUMEDGES", 1)

local w_fit = Param("w_fitSqrt", float, 0)
local w_reg = Param("w_regSqrt", float, 1)
local w_rot = Param("w_rotSqrt", float, 2)
local Offset      = Unknown("Offset", opt_float3, {N}, 3)
local RotMatrix   = Unknown("RotMatrix", opt_float9, {N}, 4)   -- row-major 3x3
local UrShape     = Image("UrShape", opt_float3, {N}, 5)
local Constraints = Image("Constraints", opt_float3, {N}, 6)   -- x < -999999.9: no handle
local G = Graph("G", {NUMEDGES}, "v0", {N}, 8, "v1", {N}, 9)
UsePreconditioner(true)

local has_target = greatereq(Constraints(0)(0), -999999.9)
Energy(Select(has_target, w_fit * (Offset(0) - Constraints(0)), 0))

-- orthonormal columns
local M = RotMatrix(0)
local col = { Vector(M(0), M(3), M(6)), Vector(M(1), M(4), M(7)), Vector(M(2), M(5), M(8)) }
Energy(w_rot * Dot3(col[1], col[2]))
Energy(w_rot * Dot3(col[1], col[3]))
Energy(w_rot * Dot3(col[2], col[3]))
for k = 1, 3 do
    Energy(w_rot * (Dot3(col[k], col[k]) - 1))
end

local predicted = Matrix3x3Mul(RotMatrix(G.v0), UrShape(G.v1) - UrShape(G.v0))
Energy(w_reg * ((Offset(G.v1) - Offset(G.v0)) - predicted))
