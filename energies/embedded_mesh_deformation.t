-- Embedded deformation: deformation-graph nodes carry an affine 3x3 matrix kept close to
-- a rotation (orthonormal columns) and predict their neighbours' displacements through
-- it; handle nodes are pulled to targets. Declaration indices follow the reference
-- example (examples/embedded_mesh_deformation).
local nv, ne = Dim("N", 0), Dim("NUMEDGES", 1)

local handleW = Param("w_fitSqrt", float, 0)
local smoothW = Param("w_regSqrt", float, 1)
local orthoW  = Param("w_rotSqrt", float, 2)
local t  = Unknown("Offset", opt_float3, {nv}, 3)
local Mx = Unknown("RotMatrix", opt_float9, {nv}, 4)   -- row-major 3x3
local g0 = Image("UrShape", opt_float3, {nv}, 5)
local q  = Image("Constraints", opt_float3, {nv}, 6)
local E  = Graph("G", {ne}, "v0", {nv}, 8, "v1", {nv}, 9)
UsePreconditioner(true)

local pinned = greatereq(q(0)(0), -999999.9)
Energy(Select(pinned, handleW * (t(0) - q(0)), 0))

local A = Mx(0)
local function column(k) return Vector(A(k), A(k + 3), A(k + 6)) end
local a1, a2, a3 = column(0), column(1), column(2)
for _, pair in ipairs({ {a1, a2}, {a1, a3}, {a2, a3} }) do
    Energy(orthoW * Dot3(pair[1], pair[2]))
end
for _, col in ipairs({ a1, a2, a3 }) do
    Energy(orthoW * (Dot3(col, col) - 1))
end

Energy(smoothW * ((t(E.v1) - t(E.v0)) - Matrix3x3Mul(Mx(E.v0), g0(E.v1) - g0(E.v0))))
