-- Cotangent-weighted mesh smoothing (same energy as the reference's
-- examples/cotangent_mesh_smoothing; same declaration indices). Every directed edge
-- v0 -> v1 carries the two vertices opposite to it (v2, v3); its Laplacian weight is the
-- mean of the cotangents at v2 and v3, recomputed from the current positions.
local N = Dim("N", 0)
local NUMEDGES = Dim("NUMEDGES", 1)

local w_fit = Param("w_fit", float, 0)
local w_reg = Param("w_reg", float, 1)
local X = Unknown("X", opt_float3, {N}, 2)          -- smoothed positions
local A = Array("A", opt_float3, {N}, 3)            -- input positions
local G = Graph("G", {NUMEDGES}, "v0", {N}, 5, "v1", {N}, 6, "v2", {N}, 7, "v3", {N}, 8)
UsePreconditioner(true)

-- cot of the angle between u and v, guarded against degenerate triangles
local function cotangent(u, v)
    local uv = Dot3(u, v)
    local sin2 = Dot3(u, u) * Dot3(v, v) - uv * uv
    sin2 = Select(greater(sin2, 0.0), sin2, 0.0001)
    return Dot3(u, v) / Sqrt(sin2)
end

Energy(w_fit * (X(0) - A(0)))

local ea = normalize(X(G.v0) - X(G.v2))
local eb = normalize(X(G.v1) - X(G.v2))
local ec = normalize(X(G.v0) - X(G.v3))
local ed = normalize(X(G.v1) - X(G.v3))
local weight = 0.5 * (cotangent(ea, eb) + cotangent(ec, ed))
weight = Sqrt(Select(greater(weight, 0.0), weight, 0.0001))
Energy(w_reg * weight * (X(G.v1) - X(G.v0)))
