-- Mesh fairing with cotangent weights, recomputed from the current positions. Each
-- directed edge (from -> to) lists the two vertices opposite to it (left, right); its
-- weight is the mean cotangent of the angles there. Declaration indices follow the
-- reference example (examples/cotangent_mesh_smoothing).
local nv, ne = Dim("N", 0), Dim("NUMEDGES", 1)

local dataW = Param("w_fit", float, 0)
local fairW = Param("w_reg", float, 1)
local P = Unknown("X", opt_float3, {nv}, 2)
local P0 = Array("A", opt_float3, {nv}, 3)
local E = Graph("G", {ne}, "v0", {nv}, 5, "v1", {nv}, 6, "v2", {nv}, 7, "v3", {nv}, 8)
UsePreconditioner(true)

local function cot_between(u, v)
    local d = Dot3(u, v)
    local s2 = Dot3(u, u) * Dot3(v, v) - d * d     -- |u x v|^2
    s2 = Select(greater(s2, 0.0), s2, 0.0001)
    return Dot3(u, v) / Sqrt(s2)
end

local function spoke(a, b) return normalize(P(a) - P(b)) end

Energy(dataW * (P(0) - P0(0)))

local w = 0.5 * (cot_between(spoke(E.v0, E.v2), spoke(E.v1, E.v2)) +
                 cot_between(spoke(E.v0, E.v3), spoke(E.v1, E.v3)))
w = Sqrt(Select(greater(w, 0.0), w, 0.0001))
Energy(fairW * w * (P(E.v1) - P(E.v0)))
